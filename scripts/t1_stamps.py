"""EXPERIMENT: per-phase wall time of T1 from s_memrealtime stamps (100 MHz) of every workgroup,
inside the production ring step (in-place update of single-lookup rows). Stamps: 0 start, 1 X + weights in LDS/regs,
2 layer 0, 3 layer 1, 4 logits, 5 dZ1, 6 dZ0, 7 dX in LDS, 15 dX stored; dedup wave: 9 passed the
barriers, 8 inserts finished."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TT_T1_DEBUG"] = os.environ.get("TT_T1_DEBUG", "8")
import torch
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep
dev = torch.device("cuda:0")
N = [50_000_000, 100_000_000]; B = 8192
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev)
g = torch.Generator(device=dev).manual_seed(1)
# the production ring over 64 resident batches (eager launches)
batches = [([torch.randint(0, n, (B,), generator=g, device=dev) for n in N],
            torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32)) for _ in range(64)]
st.capture_ring(batches, steps_per_graph=8)
nwg = B // 32
off = st.towers.nbytes - (((max(2 * nwg, 1024) * 8 + nwg * 16 * 9) * 8 + 255) // 256 * 256)
for it in range(6):
    st.run_eager(1)
    torch.cuda.synchronize()
    stm = st.towers.ws[off:off + nwg * 128].view(torch.int64).view(nwg, 16).cpu().double()
    if it < 2:
        continue
    t0 = stm[:, 0].min()
    cols = [0, 1, 2, 3, 4, 5, 6, 7, 15, 9, 8]
    rel = (stm[:, cols] - t0) * 10 / 1000  # us
    print(f"it{it} start max {float(rel[:,0].max()):.2f}us | median per stamp:",
          " ".join(f"{float(rel[:, j].median()):6.2f}" for j in range(len(cols))),
          f"| compute end max {float(rel[:, 8].max()):.2f} dedup end max {float(rel[:, 10].max()):.2f}")
