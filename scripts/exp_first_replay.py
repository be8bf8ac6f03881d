"""EXPERIMENT: host time of each ring graph's first replay against its later replays (bench.py's
run_single setup: 64 resident batches, 8-step graphs, aligned for a 20-step run after 5)."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402

num_users, num_items, D, B, layers = bench.WORKLOADS["northstar"]
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
step = FusedTwoTowerStep([num_users, num_items], [D, D], [0], [1], layers, B, dev, lr_emb=0.01, lr_dense=0.01,
                         id_dtype=torch.int64, seed=0)
batches = bench.synth_batches(num_users, num_items, B, 64, dev, "uniform", seed=1)
step.capture_ring(batches, steps_per_graph=8)
step.align_ring(20, after=5)
torch.cuda.synchronize()
pre = os.environ.get("PRE", "none")  # device activity right before the replays: none / mm / sleep
t = time.perf_counter()
if pre == "mm":
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    while time.perf_counter() - t < 0.02:
        for _ in range(10):
            a @ a
        torch.cuda.synchronize()
elif pre == "touch":  # one read per 64 KB of the tables and their state (page-walk caches warm)
    float(step.tables.weights.view(-1)[::16384].sum()) + float(step.tables.state.view(-1)[::16384].sum())
elif pre == "touch4k":  # one read per 4 KB of the tables and their state
    float(step.tables.weights.view(-1)[::1024].sum()) + float(step.tables.state.view(-1)[::1024].sum())
elif pre == "touch2m":  # one read per 2 MB
    float(step.tables.weights.view(-1)[::524288].sum()) + float(step.tables.state.view(-1)[::524288].sum())
elif pre.startswith("steps"):  # N ring steps (the bench's warm-up) right before
    step.run(int(pre[5:]))
    torch.cuda.synchronize()
elif pre.startswith("wsread"):  # read the step's workspaces (towers ws, both dedup tables) N times
    bufs = [step.towers.ws] + list(step._ring_ws()) + [step.params, step.exp_avg, step.exp_avg_sq]
    for _ in range(int(pre[6:] or 10)):
        for b_ in bufs:
            b_.view(torch.uint8).sum(dtype=torch.int64)
    torch.cuda.synchronize()
    print("ws MB", sum(b_.numel() * b_.element_size() for b_ in bufs) / 1e6, flush=True)
elif pre == "sleep":
    torch.cuda._sleep(int(2.0e9 * 0.02))
    torch.cuda.synchronize()
print(f"pre {pre}: {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
for rnd in range(3):
    ts = []
    for j in range(len(step.ring_graphs)):
        torch.cuda.synchronize()
        t = time.perf_counter()
        step.ring_graphs[j].replay()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e6)
    print(f"round {rnd}: 8-step graphs host us " + " ".join(f"{x:.0f}" for x in ts) +
          f"  (per step median {statistics.median(ts) / 8:.2f})", flush=True)
for sz, gs in sorted(step.ring_mid.items()):
    for rnd in range(2):
        ts = []
        for g in gs[:4]:
            torch.cuda.synchronize()
            t = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e6)
        print(f"{sz}-step graphs round {rnd}: " + " ".join(f"{x:.0f}" for x in ts), flush=True)
