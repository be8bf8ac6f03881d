"""EXPERIMENT: tt_pooled_fwd alone on config 5's batches (77 GB tables, B = 16,384 bags per feature of
Uniform{1..39} ids) — int64 and int32 ids, back-to-back launches timed with HIP events — against the
pooling micro (scripts/micro_pool.hip, 67 us at 5.0 TB/s) and the 123 us it took inside the step."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from two_tower_recommender_model_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
nu, ni, D, B, _ = bench.WORKLOADS["config5"]
ts = ops.TableSet([nu, ni], [D, D], [0, 1], dev)
ts.weights.zero_()
batches = bench.synth_kjt_batches(nu, ni, B, 39, 4, dev, "uniform", seed=4)
out = torch.empty(B, 2 * D, device=dev)
for dt in (torch.int64, torch.int32):
    bs = [(v.to(dt), o) for v, o, _ in batches]
    for v, o in bs:
        ts.pooled_fwd(v, o, B, out=out)
    torch.cuda.synchronize()
    n = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        v, o = bs[i % len(bs)]
        ts.pooled_fwd(v, o, B, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    nnz = sum(v.numel() for v, _ in bs) / len(bs)
    print(f"pooled_fwd {dt}: {ms * 1e3:.1f} us per launch, {nnz * 512 / ms / 1e6:.0f} GB/s of rows ({nnz:.0f} lookups)",
          flush=True)
