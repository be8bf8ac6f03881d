"""T1 (gather) with and without the dedup wave's inserts; kernel durations from rocprofv3."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

dev = torch.device("cuda:0")
N = [50_000_000, 100_000_000]
B = 8192
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev)
g = torch.Generator(device=dev).manual_seed(1)
cols = [torch.randint(0, n, (B,), generator=g, device=dev) for n in N]
lab = torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32)
st.load_batch(cols, lab)
tabs = [st.tables.table_view(0), st.tables.table_view(1)]
for mode in ("nodedup", "dedup") * 2:
    for _ in range(20):
        st.towers.fwd_bwd_gather(st.cols, st.num_embeddings, tabs, st.gpooled, st.params, st.labels, st.logits,
                                 dedup=st.tables if mode == "dedup" else None)
        if mode == "dedup":
            st.tables.dedup_rowwise_adagrad(st.gpooled, B, 0.0, 1e-10)
    torch.cuda.synchronize()
print("done")
