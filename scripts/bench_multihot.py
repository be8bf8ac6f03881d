#!/usr/bin/env python3
"""Multi-hot embedding path at SURVEY 8(d) config 5 sizes on one MI355X (KJT form):
pooled forward (tt_pooled_fwd), backward prepare (hash + scan + scatter: tt_bwd_prepare) and the
fused row-wise Adagrad (tt_bwd_rowwise_adagrad). Per-launch device time from HIP events around
graph-captured back-to-back launches; algorithmic bytes per SURVEY 8(d).

    python scripts/bench_multihot.py [--B 16384] [--D 128] [--users 50e6] [--items 100e6] [--ids uniform|zipf]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from two_tower_recommender_model_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=16384)
ap.add_argument("--D", type=int, default=128)
ap.add_argument("--users", type=float, default=50e6)
ap.add_argument("--items", type=float, default=100e6)
ap.add_argument("--maxlen", type=int, default=39, help="bag lengths ~ Uniform{1..maxlen}")
ap.add_argument("--ids", default="uniform", choices=["uniform", "zipf"])
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()

dev = torch.device("cuda:0")
B, D, F = args.B, args.D, 2
N = [int(args.users), int(args.items)]
ts = ops.TableSet(N, [D, D], [0, 1], dev)
ts.init_uniform_(torch.Generator(device=dev).manual_seed(0))
g = torch.Generator(device=dev).manual_seed(4)
lengths = torch.randint(1, args.maxlen + 1, (F * B,), generator=g, device=dev, dtype=torch.int32)
offsets = torch.zeros(F * B + 1, dtype=torch.int32, device=dev)
offsets[1:] = torch.cumsum(lengths, 0)
nnz_f = [int(lengths[f * B:(f + 1) * B].sum()) for f in range(F)]
vals = []
for f in range(F):
    if args.ids == "uniform":
        vals.append(torch.randint(0, N[f], (nnz_f[f],), generator=g, device=dev))
    else:  # Zipf s=1.05 over permuted ranks
        u = torch.rand(nnz_f[f], generator=g, device=dev, dtype=torch.float64)
        r = torch.floor(torch.pow(1.0 - u, -1.0 / 0.05)).clamp(max=N[f] - 1).to(torch.int64)
        vals.append((r * 2654435761) % N[f])
values = torch.cat(vals).contiguous()
nnz = values.numel()
keys = torch.cat([vals[0], vals[1] + (1 << 40)])
U = int(torch.unique(keys).numel())
out = torch.empty(B, F * D, dtype=torch.float32, device=dev)
gout = torch.randn(B, F * D, generator=g, device=dev) * 1e-3


def prep():
    ts.bwd_prepare(values, offsets, B, max_lookups=nnz)


def fwd():
    ts.pooled_fwd(values, offsets, B, out=out)


def upd():
    ts.bwd_rowwise_adagrad(gout, offsets, B, 0.01, 1e-10)


def timed(fns, iters):
    st = torch.cuda.current_stream()
    for f in fns:
        f()
    torch.cuda.synchronize()
    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in fns]
           for _ in range(iters)]
    for it in range(iters):
        for (a, b), f in zip(evs[it], fns):
            a.record(st)
            f()
            b.record(st)
    torch.cuda.synchronize()
    return [sum(evs[it][k][0].elapsed_time(evs[it][k][1]) for it in range(iters)) / iters for k in range(len(fns))]


ms_prep, ms_fwd, ms_upd = timed([prep, fwd, upd], args.iters)
# per lookup 8 B id (fwd) + 4D row read; per bag 4 B length + 4D pooled write
fwd_bytes = nnz * (8 + 4 * D) + F * B * (4 + 4 * D)
# prepare: ids read (hash insert) + per-lookup index writes/reads of the segment scatter
prep_bytes = nnz * 8 + F * B * 4 + nnz * 4
# update: 8 B id (bwd) per lookup + grad-out rows read per lookup (4D) + per unique row W read+write, state r+w
upd_bytes = nnz * 4 * D + U * (8 * D + 8) + nnz * 4
emb_bytes = fwd_bytes + nnz * 8 + F * B * 4 * D + U * (8 * D + 8)  # the 8(d) formula (grad-out read once per bag)
res = {
    "workload": f"config5 KJT multi-hot: {N[1]} items x {N[0]} users, D={D}, B={B}, lengths U{{1..{args.maxlen}}}, "
                f"{args.ids} ids",
    "lookups": nnz, "unique_rows": U,
    "pooled_fwd": {"ms": ms_fwd, "bytes": fwd_bytes, "GB/s": fwd_bytes / ms_fwd / 1e6},
    "bwd_prepare": {"ms": ms_prep, "bytes": prep_bytes, "GB/s": prep_bytes / ms_prep / 1e6},
    "bwd_rowwise_adagrad": {"ms": ms_upd, "bytes": upd_bytes, "GB/s": upd_bytes / ms_upd / 1e6},
    "embedding_path": {"ms": ms_fwd + ms_prep + ms_upd, "bytes_8d": emb_bytes,
                       "GB/s": emb_bytes / (ms_fwd + ms_prep + ms_upd) / 1e6},
}
print(json.dumps(res))
