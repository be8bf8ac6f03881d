"""EXPERIMENT: per-wave stamps of the row-owned T1 (tower_rows_kernel, TT_T1_DEBUG = 8, experiment
library) inside the production ring at the north-star shape: for each point, the median over
workgroups of each wave's stamp (us from the workgroup's first wave start). Points: 0 start, 1 loads
issued, 2 loads landed, 3 past barrier 1, 4 layer 0, 5 layer 1 (+ exchange write), 6 X / h strips,
7 past barrier 2, 8 logit + dZ1, 9 dZ0, 10 dX, 11 row update / dX stores, 12 dZ strips, 13 bias sums,
14 past barrier 3, 15 end."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TT_T1_DEBUG"] = str(8 | int(os.environ.get("T1_ABLATE", "0")))  # + ablation bits (16: no image, 32: no rows)
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
graph = os.environ.get("GRAPH") == "1"  # the last step of an 8-step graph replay instead of an eager step
for it in range(4):
    if graph:
        st.run(8)
    else:
        st.run_eager(1)
    torch.cuda.synchronize()
    if it < 3:
        continue
    w = st.towers.ws[off:off + dbg_bytes].view(torch.int64)[8192:8192 + nwg * 16 * 9].view(nwg, 16, 9).cpu().double()
    extra = w[:, :4, 4:8]
    w = w[:, :, :4]
    t0 = w[:, 0, :].min(dim=1, keepdim=True).values
    rel = (w - t0.unsqueeze(1)) / 100.0
    print("point   w0(q,h0) w1(q,h1) w2(c,h0) w3(c,h1)   max   (us from the workgroup's first wave start)")
    for k in range(16):
        med = rel[:, k, :].median(dim=0).values
        mx = rel[:, k, :].max(dim=1).values.median()
        print(f"  {k:3d}  " + " ".join(f"{float(x):8.2f}" for x in med) + f"  {float(mx):6.2f}")
    ex = (extra - t0.unsqueeze(1)) / 100.0
    for k, what in enumerate(["G^2 sums", "step + LDS write-back", "row stores issued", "state / dX stores"]):
        print(f"  u{k} {what:24s}" + " ".join(f"{float(x):8.2f}" for x in ex[:, k, :].median(dim=0).values))
    tmin = w[:, 0, :].min()
    print("launch span (us from the first workgroup's start): last start %.2f, end p50 %.2f, last end %.2f" % (
        float((w[:, 0, :].max() - tmin) / 100), float(((w[:, 15, :].max(dim=1).values - tmin) / 100).median()),
        float((w[:, 15, :].max() - tmin) / 100)))
    print("workgroup start spread (us, p50 / max):",
          float(((t0 - t0.min()) / 100).median()), float(((t0 - t0.min()) / 100).max()))
