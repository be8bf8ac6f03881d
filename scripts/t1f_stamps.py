"""EXPERIMENT: phase stamps of the fused T3 + T1 launch (tower_rows_t3_kernel, TT_T1_DEBUG = 8,
experiment library) in the north-star ring, a step with a pending update: per point the median over
workgroups (us from the workgroup's first wave start) and the spread over workgroups of the absolute
times (us from the launch's first stamp). Points: 0 start, F4 T3 loads issued, F5 stores drained,
F8 arrive (wave 0), F6 poll done (wave 0), F7 past the barrier, 2 image + rows landed, 3 past barrier 1,
15 end."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TT_T1_DEBUG"] = "8"
os.environ["TT_EXPERIMENT_LIB"] = "1"
import torch  # noqa: E402

from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402

dev = torch.device("cuda:0")
N, B = [50_000_000, 100_000_000], 8192
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev)
assert st.t1_fuse()
g = torch.Generator(device=dev).manual_seed(1)
batches = [([torch.randint(0, n, (B,), generator=g, device=dev) for n in N],
            torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32)) for _ in range(8)]
st.capture_ring(batches, steps_per_graph=2)
nwg = B // 32
dbg_bytes = (max(2 * nwg, 1024) * 8 + nwg * 16 * 9) * 8
off = st.towers.nbytes - ((dbg_bytes + 255) // 256 * 256)
st.run_eager(2, flush=False)
for it in range(3):
    st.run_eager(1, flush=False)
    torch.cuda.synchronize()
    w = st.towers.ws[off:off + dbg_bytes].view(torch.int64)[8192:8192 + nwg * 16 * 9].view(nwg, 16, 9).cpu().double()
    t0 = w[:, 0, :4].min(dim=1, keepdim=True).values  # per workgroup
    g0 = float(t0.min())
    pts = [("0 start", w[:, 0, 0]), ("F4 T3 loads issued", w[:, 4, 4]), ("F5 stores drained", w[:, 5, 4]),
           ("F8 arrive", w[:, 8, 4]), ("F6 poll done", w[:, 6, 4]), ("F7 past barrier", w[:, 7, 4]),
           ("2 image+rows landed", w[:, 2, 0]), ("3 past barrier 1", w[:, 3, 0]), ("15 end", w[:, 15, 0])]
    print(f"step {it}: point                 rel p50   abs p10   abs p50   abs p90   abs max  (us)")
    for name, v in pts:
        rel = (v - t0[:, 0]) / 100.0
        ab = (v - g0) / 100.0
        q = torch.quantile(ab, torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64))
        print(f"  {name:24s} {float(rel.median()):8.2f} {float(q[0]):9.2f} {float(q[1]):9.2f} {float(q[2]):9.2f} "
              f"{float(ab.max()):9.2f}")
st.flush()
torch.cuda.synchronize()
print("timeouts", st.fuse_timeouts())
