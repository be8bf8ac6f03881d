"""Diagnostic: north-star step time under stream / graph-granularity variants, and the host time
spent inside the graph-replay calls. Not part of the product or the tests.

    python scripts/step_probe.py [--workload northstar]
"""
import argparse
import gc
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="northstar")
ap.add_argument("--steps", type=int, default=64)
ap.add_argument("--variants", default="11:1,00:1,00:8,11:8,10:8,01:8")
args = ap.parse_args()

num_users, num_items, D, B, layers = bench.WORKLOADS[args.workload]
dev = torch.device("cuda:0")
batches = bench.synth_batches(num_users, num_items, B, 8, dev, "uniform", seed=1)
for v in args.variants.split(","):
    flags, k = v.split(":")
    k = int(k)
    step = FusedTwoTowerStep([num_users, num_items], [D, D], [0], [1], layers, B, dev, id_dtype=torch.int64,
                             overlap_prepare=flags[0] == "1", overlap_towers=flags[1] == "1")
    step.capture_pool(batches, steps_per_graph=k)
    n = len(step.pool_graphs)
    for i in range(2 * n):
        step.replay(i)
    torch.cuda.synchronize()
    reps = max(1, args.steps // k)
    t0 = time.perf_counter()
    for i in range(reps):
        step.replay(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    us = (t2 - t0) / (reps * k) * 1e6
    host = (t1 - t0) / (reps * k) * 1e6
    print(f"overlap_prepare={flags[0]} overlap_towers={flags[1]} steps/graph={k}: {us:7.2f} us/step "
          f"(host in replay {host:6.2f} us/step), loss {float(step.loss):.4f}", flush=True)
    del step
    gc.collect()
    torch.cuda.empty_cache()
