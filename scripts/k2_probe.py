"""EXPERIMENT: K2 role breakdown — T2 alone (tower_wgrad_kernel), the fused row-wise Adagrad alone
(dd_adagrad_kernel) and the combined launch (tower_wgrad_dedup_kernel), north-star shapes.
Run under `rocprofv3 --kernel-trace --stats` and read the per-kernel averages."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

dev = torch.device("cuda:0")
N = [50_000_000, 100_000_000]; B = 8192
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev)
g = torch.Generator(device=dev).manual_seed(1)
st.load_batch([torch.randint(0, n, (B,), generator=g, device=dev) for n in N],
              torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32))
tabs = [st.tables.table_view(0), st.tables.table_view(1)]
for _ in range(20):
    st.towers.fwd_bwd_gather(st.cols, st.num_embeddings, tabs, st.gpooled, st.params, st.labels, st.logits,
                             dedup=st.tables, dedup_tables=(0, 1))
    st.towers.wgrad(st.loss)
    st.tables.dedup_resolve()
    st.tables.dedup_rowwise_adagrad(st.gpooled, B, st.lr_emb, st.eps)
    st.towers.update(st.params, st.exp_avg, st.exp_avg_sq, st.adam_state, lr=st.lr_dense)
for _ in range(20):
    st.step()
torch.cuda.synchronize()
print("done")
