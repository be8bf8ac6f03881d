"""Where the driver-form bench line's fixed cost goes (experiment, not a test).

`bench.py --steps 20 --warmup 5` reads ~1.5 us a step above the default 50-step line: a fixed
~50 us per timed run spread over 20 steps. This replays the north-star ring as bench.py's
run_single does and times many 20-step runs three ways at once: the host clock (what the line
reports), HIP events on the replay stream around the run (device time, first kernel's queueing
included) and the host time until the first graph launch returns. Variants of how the 20 steps
are grouped into graph launches:
  cur    bench.py's grouping (remainder 4 first, then 8 + 8)
  r1     a single-step graph first, then the rest as cur would group 19
  r2     two single-step graphs first
Usage (GPU): python scripts/exp_driver_overhead.py [--trials 12]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=12)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--idle", type=float, default=0.0, help="seconds of host sleep after each run")
    ap.add_argument("--variants", default="cur,r1,r2")
    ap.add_argument("--prewarm", type=int, default=16, help="steps replayed once before the trials")
    ap.add_argument("--sweep", default="none", choices=["none", "page", "frag", "pf", "busy", "busyread"],
                    help="before anything: read one float per 4 KB page / per 2 MB of the tables")
    ap.add_argument("--perstep", type=int, default=0, help="first: this many single-step graphs, timed each")
    ap.add_argument("--passes", type=int, default=None, help="TableSet.prefault passes (default: the library's)")
    a = ap.parse_args()
    if a.passes is not None:
        from two_tower_recommender_model_amd import ops
        ops.TableSet.prefault.__defaults__ = (4096, a.passes)
    num_users, num_items, D, B, layers = bench.WORKLOADS["northstar"]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    step = FusedTwoTowerStep([num_users, num_items], [D, D], [0], [1], layers, B, dev, lr_emb=0.01,
                             lr_dense=0.01, id_dtype=torch.int64, seed=0)
    batches = bench.synth_batches(num_users, num_items, B, 64, dev, "uniform", seed=1)
    step.capture_ring(batches, steps_per_graph=8)
    if a.sweep != "none":
        w = step.tables.weights.view(-1)
        stride = 1024 if a.sweep == "page" else 512 * 1024
        t0 = time.perf_counter()
        if a.sweep == "pf":
            step.tables.prefault()
            x = 0.0
        elif a.sweep == "busy":  # ~10 ms of MFMA work touching no table
            m = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
            for _ in range(20):
                m2 = m @ m
            x = float(m2[0, 0])
        elif a.sweep == "busyread":  # ~10 ms of streaming reads of 4 GB (not the tables)
            m = torch.ones(1 << 30, device=dev)
            x = 0.0
            for _ in range(16):
                x += float(m.sum())
        else:
            x = float(w[::stride].sum()) + float(step.tables.state.view(-1)[::stride].sum())
        torch.cuda.synchronize()
        print(f"sweep {a.sweep}: {(time.perf_counter() - t0) * 1e3:.1f} ms ({x:.3g})", flush=True)
    if a.perstep:
        ts = []
        for _ in range(a.perstep):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            step.run(1)
            e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        print("per-step device us: " + " ".join(f"{x.elapsed_time(y) * 1e3:.1f}" for x, y in ts), flush=True)
    if a.prewarm:
        step.run(a.prewarm)
    torch.cuda.synchronize()
    res = {}
    K, W = a.steps, a.warmup
    for t in range(a.trials):
        for v in a.variants.split(","):
            lead = {"cur": 0, "r1": 1, "r2": 2}[v]
            step.align_ring(K - lead, after=W + lead)
            step.run(W)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            for _ in range(lead):
                step.run(1)
            t1 = time.perf_counter()
            step.run(K - lead)
            e1.record()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res.setdefault(v, []).append((dt * 1e6 / K, e0.elapsed_time(e1) * 1e3 / K, (t1 - t0) * 1e6))
            if a.idle:
                time.sleep(a.idle)
        print(f"trial {t}: " + " ".join(f"{v} {r[-1][0]:.2f}/{r[-1][1]:.2f}" for v, r in res.items()), flush=True)
    for v, rows in res.items():
        rows = sorted(rows)
        med = rows[len(rows) // 2]
        print(f"{v:4s} host us/step min {rows[0][0]:.2f} med {med[0]:.2f} | device us/step (same run) "
              f"{med[1]:.2f} | lead launches {med[2]:.1f} us", flush=True)


if __name__ == "__main__":
    main()
