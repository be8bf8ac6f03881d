"""EXPERIMENT (experiment library): per-phase wall time of the ring tail's weight-gradient tiles
(wgrad_lds_block_rm) from s_memrealtime stamps (100 MHz): 0 start, 1 first chunk in LDS (the
slice's operand loads landed), 2 MFMAs done, 3 slab stored. The tail's grid: [0, n_ins) insert
workgroups, then 192 tile workgroups, then the bias / loss workgroups, then the slot workgroups."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TT_T2_STAMPS"] = "1"
os.environ["TT_EXPERIMENT_LIB"] = "1"
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
INS_PT = 1
n_ins = -(-(-(-2 * B // (256 * INS_PT))) // 8) * 8
ntile = 6 * 32
nbias = (2 * (128 + 64) + 1 + 3) // 4
for it in range(6):
    st.run_eager(1)
    torch.cuda.synchronize()
    if it < 2:
        continue
    stm = st.towers.ws[off:off + dbg_bytes].view(torch.int64)[:(n_ins + ntile + nbias) * 8]
    stm = stm.view(-1, 8).cpu().double()[n_ins:]
    t0 = stm[:ntile, 0].min()
    rel = (stm[:, :4] - t0) / 100.0
    tl, bs = rel[:ntile], rel[ntile:]
    md = lambda x: float(x.median())  # noqa: E731
    print(f"it{it}: tiles start p50 {md(tl[:, 0]):.2f} max {float(tl[:, 0].max()):.2f} | loads {md(tl[:, 1] - tl[:, 0]):.2f} "
          f"(max {float((tl[:, 1] - tl[:, 0]).max()):.2f}) | mfma {md(tl[:, 2] - tl[:, 1]):.2f} | store "
          f"{md(tl[:, 3] - tl[:, 2]):.2f} | end p50 {md(tl[:, 3]):.2f} max {float(tl[:, 3].max()):.2f} || bias start p50 "
          f"{md(bs[:, 0]):.2f} end max {float(bs[:, 3].max()):.2f}", flush=True)
