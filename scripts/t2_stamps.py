"""EXPERIMENT: per-phase wall time of T2 (staged tower weight gradients) from s_memrealtime stamps
(100 MHz): 0 start, 1 first chunk in LDS (all operand loads landed), 2 MFMAs done, 3 slab stored.
Bias workgroups (after the tile workgroups) stamp 0 and 3."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TT_T2_STAMPS"] = "1"
import torch
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

dev = torch.device("cuda:0")
N = [50_000_000, 100_000_000]; B = 8192
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev)
g = torch.Generator(device=dev).manual_seed(1)
# the production ring (T2 = tower_wgrad_insert_kernel: tiles first, then bias, then inserts)
batches = [([torch.randint(0, n, (B,), generator=g, device=dev) for n in N],
            torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32)) for _ in range(64)]
st.capture_ring(batches, steps_per_graph=8)
nres = 0
ntile = 6 * 32
nbias = (2 * (128 + 64) + 1 + 3) // 4
nwg = nres + ntile + nbias
off = st.towers.nbytes - (((max(2 * (B // 32), 1024) * 8 + (B // 32) * 16 * 9) * 8 + 255) // 256 * 256)
for it in range(6):
    st.run_eager(1)
    torch.cuda.synchronize()
    stm = st.towers.ws[off:off + nwg * 64].view(torch.int64).view(nwg, 8).cpu().double()
    if it < 2:
        continue
    stm = stm[nres:]
    t0 = stm[:, 0].min()
    rel = (stm[:, :4] - t0) * 10 / 1000
    tl, bs = rel[:ntile], rel[ntile:]
    md = lambda x: float(x.median())  # noqa: E731
    print(f"it{it}: tiles start p50 {md(tl[:, 0]):.2f} max {float(tl[:, 0].max()):.2f} | loads {md(tl[:, 1] - tl[:, 0]):.2f} "
          f"| mfma {md(tl[:, 2] - tl[:, 1]):.2f} | store {md(tl[:, 3] - tl[:, 2]):.2f} | end p50 {md(tl[:, 3]):.2f} "
          f"max {float(tl[:, 3].max()):.2f} || bias start p50 {md(bs[:, 0]):.2f} end max {float(bs[:, 3].max()):.2f}")
