"""EXPERIMENT: per-phase wall time of T1 from s_memrealtime stamps (100 MHz) of every workgroup."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TT_T1_DEBUG"] = os.environ.get("TT_T1_DEBUG", "8")
import torch
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep
dev = torch.device("cuda:0")
N = [50_000_000, 100_000_000]; B = 8192
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev)
g = torch.Generator(device=dev).manual_seed(1)
st.load_batch([torch.randint(0, n, (B,), generator=g, device=dev) for n in N], torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32))
tabs = [st.tables.table_view(0), st.tables.table_view(1)]
nwg = B // 32
off = st.towers.nbytes - ((nwg * 128 + 255) // 256 * 256)
for it in range(6):
    st.towers.fwd_bwd_gather(st.cols, st.num_embeddings, tabs, st.gpooled, st.params, st.labels, st.logits,
                             dedup=st.tables if os.environ.get("DEDUP") else None)
    if os.environ.get("DEDUP"):
        st.tables.dedup_rowwise_adagrad(st.gpooled, B, 0.0, 1e-10)
    torch.cuda.synchronize()
    stm = st.towers.ws[off:off + nwg * 128].view(torch.int64).view(nwg, 16).cpu().double()
    if it < 2:
        continue
    t0 = stm[:, 0].min()
    cols = [0, 1, 2, 3, 4, 5, 6, 7, 15]
    rel = (stm[:, cols] - t0) * 10 / 1000  # us
    print(f"it{it} start spread {float(rel[:,0].max()):.2f}us | median per stamp:",
          " ".join(f"{float(rel[:, j].median()):6.2f}" for j in range(len(cols))),
          f"| last end {float(rel[:, -1].max()):.2f}")
