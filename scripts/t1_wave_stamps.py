"""EXPERIMENT: per-wave barrier arrivals in T1 (TT_T1_DEBUG = 8 | 64) inside the production ring:
for each of the 7 barriers, the median over workgroups of each wave's arrival, relative to the
workgroup's previous barrier (the last arrival there); waves 0-3 = query tower, 4-7 = candidate
tower, 8 = the dedup wave. Tells which waves set each phase's length."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# extra TT_T1_DEBUG bits from argv[1]: 4 = every lookup reads row 0, 32 = no id load (id 1),
# 2 = no dX store, 128 = no in-place row / state store
os.environ["TT_T1_DEBUG"] = str(72 | (int(sys.argv[1]) if len(sys.argv) > 1 else 0))
import torch  # noqa: E402

from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402

dev = torch.device("cuda:0")
N, B = [50_000_000, 100_000_000], 8192
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev)
g = torch.Generator(device=dev).manual_seed(1)
batches = [([torch.randint(0, n, (B,), generator=g, device=dev) for n in N],
            torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32)) for _ in range(64)]
st.capture_ring(batches, steps_per_graph=8)
nwg = B // 32
dbg_bytes = (max(2 * nwg, 1024) * 8 + nwg * 16 * 9) * 8
off = st.towers.nbytes - ((dbg_bytes + 255) // 256 * 256)
for it in range(4):
    st.run_eager(1)
    torch.cuda.synchronize()
    if it < 3:
        continue
    w = st.towers.ws[off:off + dbg_bytes].view(torch.int64)[8192:8192 + nwg * 16 * 9].view(nwg, 16, 9).cpu().double()
    w = w[:, :15, :]  # points 0..8, 9 = past barrier 7, 10 = first dX / row store issued,
    # 11 = phase 1 after the X^T strip, 12 = after layer 0's MFMA, 13 = after the W0 image, 14 = phase 5 after its MFMA
    t0 = w[:, 0, :].min(dim=1, keepdim=True).values  # workgroup start
    rel = (w - t0.unsqueeze(1)) / 100.0  # us, [wg, point, wave]
    print(f"it{it}: arrival (us from the workgroup's first wave start), median over workgroups")
    print("  point  " + " ".join(f"  w{j}" for j in range(9)) + "   last  phase")
    prev = torch.zeros(nwg, dtype=torch.float64)
    for k in [0, 1, 11, 12, 13, 2, 3, 4, 5, 14, 6, 7, 9, 10, 8]:
        med = rel[:, k, :].median(dim=0).values
        last = rel[:, k, :].max(dim=1).values
        ph = float((last - prev).median())
        print(f"  {k:5d}  " + " ".join(f"{float(x):5.2f}" for x in med) + f"  {float(last.median()):5.2f}  {ph:5.2f}")
        prev = last
