"""EXPERIMENT: config 2's tables and towers (10M items x 5M users, D = 64, towers [128, 64]) on the
production ring at B = 4096 (the BASELINE batch: 128 T1 tiles, half the CUs) and B = 8192 (256
tiles, every CU): if the step is a per-tile latency chain, doubling the tiles costs little time —
the price of giving B = 4096 all 256 CUs with 16-row tiles is bounded by this."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402

num_users, num_items, D, _, layers = bench.WORKLOADS["config2"]
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
for B in (4096, 8192, 4096, 8192):
    step = FusedTwoTowerStep([num_users, num_items], [D, D], [0], [1], layers, B, dev, lr_emb=0.01, lr_dense=0.01,
                             id_dtype=torch.int64, seed=0)
    batches = bench.synth_batches(num_users, num_items, B, 64, dev, "uniform", seed=1)
    step.capture_ring(batches, steps_per_graph=8)
    K, W = 96, 32
    step.align_ring(K, after=W)
    step.run(W)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step.run(K)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"config2 tables, B {B}: {dt / K * 1e6:.2f} us/step, {K * B / dt / 1e6:.1f} M pairs/s", flush=True)
    del step, batches
    torch.cuda.empty_cache()
