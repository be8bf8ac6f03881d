"""Does the tables' allocation (its page fragments) move the north-star step? (experiment, not a test)

The first-run study (profiles/r06dr_*, r06pf*) showed the step's random row gathers pay page-table
walks. This builds the north-star ring over tables allocated three ways and times warm runs:
  torch       the caching allocator (what the product uses)
  contiguous  hipExtMallocWithFlags(hipDeviceMallocContiguous): one physically contiguous range,
              so the driver can map it with the largest fragments
Usage (GPU): python scripts/exp_table_alloc.py --alloc torch|contiguous [--runs 5 --steps 200]
"""
import argparse
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from two_tower_recommender_model_amd import ops  # noqa: E402
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402
from two_tower_recommender_model_amd.sharded import _DeviceArray  # noqa: E402

HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--alloc", default="torch", choices=["torch", "contiguous"])
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--workload", default="northstar")
    ap.add_argument("--min-bytes", type=int, default=None, help="ops.TABLE_ALLOC_MIN_BYTES for this run")
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    num_users, num_items, D, B, layers = bench.WORKLOADS[a.workload]
    if a.min_bytes is not None:
        ops.TABLE_ALLOC_MIN_BYTES = a.min_bytes
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    Ns = [num_users, num_items]
    weights = None
    if a.alloc == "torch":  # every TableSet buffer from the caching allocator (the state too)
        ops.TABLE_ALLOC_MIN_BYTES = 1 << 62
    if a.alloc == "contiguous":
        hip = C.CDLL("libamdhip64.so")
        n = sum(Ns) * D
        p = C.c_void_p()
        t0 = time.perf_counter()
        rc = hip.hipExtMallocWithFlags(C.byref(p), C.c_size_t(n * 4), C.c_uint(HIP_DEVICE_MALLOC_CONTIGUOUS))
        print(f"hipExtMallocWithFlags(contiguous, {n * 4 / 1e9:.1f} GB): rc {rc} in {time.perf_counter() - t0:.2f} s",
              flush=True)
        if rc != 0:
            sys.exit(3)
        raw = torch.as_tensor(_DeviceArray(p.value, n * 4), device=dev)
        weights = raw.view(torch.float32)
    ts = ops.TableSet(Ns, [D, D], [0, 1], dev, weights=weights)
    ts.init_uniform_(torch.Generator(device=dev).manual_seed(0))
    step = FusedTwoTowerStep(Ns, [D, D], [0], [1], layers, B, dev, lr_emb=0.01, lr_dense=0.01,
                             id_dtype=torch.int64, seed=0, tables=ts)
    batches = bench.synth_batches(num_users, num_items, B, 64, dev, "uniform", seed=1)
    step.capture_ring(batches, steps_per_graph=8)
    step.run(64)
    torch.cuda.synchronize()
    res = []
    for _ in range(a.runs):
        t0 = time.perf_counter()
        step.run(a.steps)
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) / a.steps * 1e6)
    print(f"{a.alloc}: us/step " + " ".join(f"{x:.2f}" for x in res) + f" | loss {float(step.loss):.6f}", flush=True)


if __name__ == "__main__":
    main()
