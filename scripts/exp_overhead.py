"""EXPERIMENT: the fixed host cost around a timed ring run (bench.py run_single's region: sync, K
steps of graph replays, sync). dt(K) = fixed + K * step: fits the intercept from several K and
splits it with HIP events into "GPU busy" and "host around it" (the first launch's latency and the
final synchronize's wake-up). Env knobs to try are set by the caller (e.g. HIP_FORCE_DEV_KERNARG);
TT_SPIN=1 asks HIP for spin waits (hipSetDeviceFlags(hipDeviceScheduleSpin)) before torch's
first device call."""
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if os.environ.get("TT_SPIN") == "1":
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(ctypes.c_uint(1)), flush=True)

import torch  # noqa: E402

import bench  # noqa: E402
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402


def main():
    num_users, num_items, D, B, layers = bench.WORKLOADS["northstar"]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    step = FusedTwoTowerStep([num_users, num_items], [D, D], [0], [1], layers, B, dev, lr_emb=0.01,
                             lr_dense=0.01, id_dtype=torch.int64, seed=0)
    k = int(os.environ.get("TT_SPG", "8"))
    batches = bench.synth_batches(num_users, num_items, B, 32, dev, "uniform", seed=1)
    step.capture_ring(batches, steps_per_graph=k)
    lat = []
    for _ in range(200):
        t = time.perf_counter()
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t)
    x = torch.zeros(1, device=dev)
    kl = []
    for _ in range(200):
        torch.cuda.synchronize()
        t = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        kl.append(time.perf_counter() - t)
    print(f"idle sync {statistics.median(lat) * 1e6:.1f} us; tiny kernel launch+sync "
          f"{statistics.median(kl) * 1e6:.1f} us", flush=True)
    rows = []
    for K in [4, 8, 12, 16, 20, 24, 32, 48, 64]:
        step.align_ring(K, after=5)
        step.run(5)
        dts, spans = [], []
        for rep in range(7):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            step.run(3)
            step.align_ring(K, after=0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a.record()
            step.run(K)
            b.record()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            dts.append(dt * 1e6)
            spans.append(a.elapsed_time(b) * 1e3)
        m, s = statistics.median(dts), statistics.median(spans)
        rows.append((K, m, s))
        print(f"K {K:3d}: host {m:8.1f} us ({m / K:6.2f}/step)  events {s:8.1f} us ({s / K:6.2f}/step)  "
              f"host-events {m - s:6.1f} us   min host {min(dts):8.1f}", flush=True)
    n = len(rows)
    mx = sum(r[0] for r in rows) / n
    for j, name in ((1, "host"), (2, "events")):
        my = sum(r[j] for r in rows) / n
        sl = sum((r[0] - mx) * (r[j] - my) for r in rows) / sum((r[0] - mx) ** 2 for r in rows)
        print(f"fit {name}: {my - sl * mx:.1f} us + K x {sl:.2f} us", flush=True)


if __name__ == "__main__":
    main()
