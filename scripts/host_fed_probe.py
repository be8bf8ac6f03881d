"""Where the host-fed pipeline's time goes (north-star shape): (1) the classic step's pool graphs
over resident batches (the kernels HostFedPipeline replays), (2) the host-fed pipeline itself,
(3) its host fill alone (numpy -> pinned copies, no device work)."""
import itertools
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402
from two_tower_recommender_model_amd.host_pipeline import HostFedPipeline, synthetic_host_batches  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
N, B, g = [50_000_000, 100_000_000], 8192, 8
step = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev, lr_emb=0.01, lr_dense=0.01, seed=0)
host = synthetic_host_batches(N, B, 64, seed=1)
pipe = HostFedPipeline(step, group=g, depth=4)
# (1) the pool graphs alone (data already in the device slots)
for gr in pipe.graphs:
    gr.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for r in range(30):
    pipe.graphs[r % 3].replay()
torch.cuda.synchronize()
print(f"classic pool graphs: {(time.perf_counter() - t0) / (30 * g) * 1e6:.1f} us/step")
# (2) host-fed
src = itertools.cycle(host)
pipe.run(src, max_steps=4 * g)
torch.cuda.synchronize()
t0 = time.perf_counter()
n = pipe.run(src, max_steps=64 * g)
torch.cuda.synchronize()
print(f"host-fed: {(time.perf_counter() - t0) / n * 1e6:.1f} us/step over {n} steps")
# (3) the host copies alone
pin = np.zeros((g, 2, B), np.int64)
t0 = time.perf_counter()
for r in range(64):
    for j in range(g):
        cols, lab = host[(r * g + j) % len(host)]
        for f, c in enumerate(cols):
            pin[j, f] = np.asarray(c)
print(f"host fill alone: {(time.perf_counter() - t0) / (64 * g) * 1e6:.1f} us/step")
