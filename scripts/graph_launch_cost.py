"""Host time of one HIP graph launch (replay) per ring graph size, and the GPU's idle gap the first
launch leaves after a synchronize (north-star shape): what a short timed region pays up front."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
N, B = [50_000_000, 100_000_000], 8192
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev)
g = torch.Generator(device=dev).manual_seed(1)
batches = [([torch.randint(0, n, (B,), generator=g, device=dev) for n in N],
            torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32)) for _ in range(16)]
st.capture_ring(batches, steps_per_graph=8)
st.run(16)
torch.cuda.synchronize()
for name, graphs in [("1", st.ring_small), ("2", st.ring_mid[2]), ("4", st.ring_mid[4]), ("8", st.ring_graphs)]:
    host, wall = [], []
    for rep in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        graphs[0].replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e6)
        wall.append((t2 - t0) * 1e6)
    print(f"{name}-step graph: launch host {sorted(host)[3]:.1f} us, launch->done {sorted(wall)[3]:.1f} us")
