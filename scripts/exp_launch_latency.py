"""EXPERIMENT: where the driver-form line's extra time goes (bench.py run_single's sequence: 64
batches, 8-step graphs aligned for K steps after W): host time until run(K) returns (the launches),
host time until the synchronize returns, and the GPU span between events recorded right before and
after the launches. MODE=plain: as bench.py; MODE=prelaunch: a trivial kernel launched and synced
right before t0 (the host launch path warm)."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402

W, K = int(os.environ.get("W", "5")), int(os.environ.get("K", "20"))
mode = os.environ.get("MODE", "plain")
num_users, num_items, D, B, layers = bench.WORKLOADS["northstar"]
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
step = FusedTwoTowerStep([num_users, num_items], [D, D], [0], [1], layers, B, dev, lr_emb=0.01, lr_dense=0.01,
                         id_dtype=torch.int64, seed=0)
batches = bench.synth_batches(num_users, num_items, B, 64, dev, "uniform", seed=1)
step.capture_ring(batches, steps_per_graph=8)
x = torch.zeros(1, device=dev)
for rep in range(4):
    step.align_ring(K, after=W)
    step.run(W)
    torch.cuda.synchronize()
    if mode == "prelaunch":
        x.add_(1)
        torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    step.run(K)
    t1 = time.perf_counter()
    b.record()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{mode} W {W} K {K} rep {rep}: launches return {(t1 - t0) * 1e6:7.1f} us, total {(t2 - t0) * 1e6:7.1f} us "
          f"({(t2 - t0) * 1e6 / K:.2f}/step), GPU span {a.elapsed_time(b) * 1e3:7.1f} us", flush=True)
