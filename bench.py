#!/usr/bin/env python3
"""Benchmark: training pairs/s of the two-tower step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload northstar|config2]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (default = BASELINE.json north star): synthetic 100M-item x 50M-user two-tower, emb_dim
128, batch 8192 per GPU, towers [128, 64], single-hot ids uniform over each table (ids kept in HBM),
labels Bernoulli(0.5), random-init weights. One "step" = the full training step: device KJT build,
pooled forward, towers fwd (bf16 MFMA), dot + BCE, towers bwd, fused dedup + row-wise Adagrad on the
tables, Adam on the towers.

N = 1: the fused step replayed as one HIP graph. N > 1: DistributedModelParallel over RCCL (the
tables row-wise sharded, towers data-parallel) — eager launches. Timing: W untimed steps, barrier +
synchronize, K timed steps, synchronize + barrier, max over ranks; rank 0 prints ONE JSON line.
Also reported: the embedding path's dominant kernel against the HBM roofline (HIP events on its
own stream) and the CPU restatement's pairs/s on this host (rank 0, N = 1, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
MFMA_BF16_PEAK_TFS = 2500.0  # dense bf16 MFMA spec (same table; the 5 PF figure assumes 2:1 sparsity)

WORKLOADS = {
    # name: (num_users, num_items, dim, batch, layer_sizes)
    "northstar": (50_000_000, 100_000_000, 128, 8192, [128, 64]),
    "config2": (5_000_000, 10_000_000, 64, 4096, [128, 64]),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="northstar", choices=sorted(WORKLOADS))
    ap.add_argument("--ids", default="uniform", choices=["uniform", "zipf"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=2_000_000, help="table rows of the CPU sample")
    ap.add_argument("--cpu-steps", type=int, default=20)
    ap.add_argument("--kernel-iters", type=int, default=50)
    ap.add_argument("--steps-per-graph", type=int, default=8, choices=[1, 2, 4, 8])
    return ap.parse_args()


def synth_batches(num_users, num_items, B, n, device, ids, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    out = []
    for _ in range(n):
        if ids == "uniform":
            u = torch.randint(0, num_users, (B,), generator=g, device=device, dtype=torch.int64)
            it = torch.randint(0, num_items, (B,), generator=g, device=device, dtype=torch.int64)
        else:  # Zipf-like (s ~ 1.05) over randomly permuted ranks: heavy hot rows
            def zipf(N):
                u01 = torch.rand(B, generator=g, device=device, dtype=torch.float64)
                r = torch.floor(torch.exp(u01 * torch.log(torch.tensor(float(N), device=device, dtype=torch.float64))))
                return ((r.to(torch.int64) * 2654435761) % N)
            u, it = zipf(num_users), zipf(num_items)
        lab = torch.randint(0, 2, (B,), generator=g, device=device, dtype=torch.int32)
        out.append(([u, it], lab))
    return out


def algorithmic_bytes(step, nnz: int, uniq: int):
    """Per-launch algorithmic bytes (SURVEY.md 8(d) accounting, per kernel):
    pooled_fwd : per lookup id (8) + row (4D); per bag offset (4) + pooled write (4D)
    adagrad k2d: per lookup bag index (4) + grad row (4D); per unique row read+write row (8D),
                 read+write state (8), segment/slot/key bookkeeping (20)."""
    D = step.dims[0]
    idb = 8 if step.id_dtype == torch.int64 else 4
    nb = step.F * step.B
    fwd = nnz * (idb + 4 * D) + nb * (4 + 4 * D)
    k2d = nnz * (4 + 4 * D) + uniq * (8 * D + 8 + 20)
    return fwd, k2d


def time_kernel(fn, iters):
    """Average device time of one fn() launch: `iters` launches captured back to back in one HIP
    graph (no host launch gaps between them), replayed between two HIP events on the stream the
    graph runs on (the current stream)."""
    st = torch.cuda.current_stream()
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream()
    cs.wait_stream(st)
    with torch.cuda.stream(cs):
        fn()  # warm (workspaces exist before capture)
        with torch.cuda.graph(g, stream=cs):
            for _ in range(iters):
                fn()
    st.wait_stream(cs)
    g.replay()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record(st)
    g.replay()
    b.record(st)
    b.synchronize()
    return a.elapsed_time(b) / iters  # ms


def cpu_baseline(args, num_users, num_items, D, B, layers):
    """The oracle (CPU restatement of TorchRec's unsharded CPU path, sparse touched-row update) on
    this host's cores, bounded sample: full B, D, towers; tables scaled to --cpu-rows rows."""
    from oracle import ref

    threads = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(threads)
    rows = min(args.cpu_rows, num_users), min(args.cpu_rows, num_items)
    st = ref.init_state(list(rows), [D, D], [0, 1], [0], [1], layers, seed=0)
    g = torch.Generator().manual_seed(0)
    batches = []
    for _ in range(4):
        cols = [torch.randint(0, rows[0], (B,), generator=g), torch.randint(0, rows[1], (B,), generator=g)]
        lab = torch.randint(0, 2, (B,), generator=g)
        v, l, o = ref.kjt_build([c.numpy() for c in cols], list(rows))
        batches.append((torch.from_numpy(v), torch.from_numpy(o), lab))
    for i in range(2):
        v, o, lab = batches[i % 4]
        ref.train_step(st, v, o, B, lab, 0.01, 0.01)
    t0 = time.perf_counter()
    n = args.cpu_steps
    for i in range(n):
        v, o, lab = batches[i % 4]
        ref.train_step(st, v, o, B, lab, 0.01, 0.01)
    dt = time.perf_counter() - t0
    return {
        "value": round(n * B / dt, 1), "unit": "pairs/s", "cores": threads, "kind": "port",
        "sample": f"{n} steps of the oracle train_step (torch CPU fp32: embedding_bag sum, towers "
                  f"{layers}, BCE, sparse row-wise Adagrad, Adam) at B={B}, D={D}, tables scaled to "
                  f"{rows[0]}x{D} / {rows[1]}x{D} rows; host CPU {platform.processor() or platform.machine()}",
    }


def run_single(args):
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    num_users, num_items, D, B, layers = WORKLOADS[args.workload]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    step = FusedTwoTowerStep([num_users, num_items], [D, D], [0], [1], layers, B, dev, lr_emb=0.01,
                             lr_dense=0.01, id_dtype=torch.int64, seed=0)
    batches = synth_batches(num_users, num_items, B, 8, dev, args.ids, seed=1)
    # HIP graphs over the 8 resident batches, k full steps per graph (no input copies): a graph
    # launch costs the host ~35-55 us, more than a step's GPU time, so k > 1 keeps the GPU fed
    # (graphs of k steps, plus single-step graphs for a remainder, so exactly K steps are timed)
    k = args.steps_per_graph
    step.capture_pool(batches, steps_per_graph=k)
    big = step.pool_graphs
    step.capture_pool(batches, steps_per_graph=1)
    small = step.pool_graphs

    def run(n, i=0):
        while n >= k:
            big[(i // k) % len(big)].replay()
            i, n = i + k, n - k
        while n > 0:
            small[i % len(small)].replay()
            i, n = i + 1, n - 1

    run(args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps_run = args.steps
    ms = dt / steps_run * 1e3
    value = steps_run * B / dt
    loss = float(step.loss)
    # ---- dominant embedding kernels vs the HBM roofline (HIP events, same stream)
    cols = batches[(args.steps - 1) % len(batches)][0]
    ne = step.num_embeddings
    keys = torch.cat([(c % n) + (t << 40) for t, (c, n) in enumerate(zip(cols, ne))])
    nz = torch.cat([c != 0 for c in cols])
    nnz = int(nz.sum())
    uniq = int(torch.unique(keys[nz]).numel())
    fwd_bytes, k2d_bytes = algorithmic_bytes(step, nnz, uniq)
    t_fwd = time_kernel(lambda: step.tables.pooled_fwd_cols(cols, ne, out=step.pooled), args.kernel_iters)
    # the fused backward re-applied to one prepared dedup (lr 0: the tables are left unchanged);
    # the op is the per-row kernel plus the hot-row kernel (idle for these ids)
    step.tables.bwd_prepare_cols(cols, ne)
    t_k2d = time_kernel(lambda: step.tables.bwd_rowwise_adagrad(step.gpooled, None, B, 0.0, 1e-10),
                        args.kernel_iters)
    kern = {
        "pooled_fwd": {"ms": round(t_fwd, 5), "bytes": fwd_bytes, "GB/s": round(fwd_bytes / t_fwd / 1e6, 1)},
        "bwd_rowwise_adagrad": {"ms": round(t_k2d, 5), "bytes": k2d_bytes, "GB/s": round(k2d_bytes / t_k2d / 1e6, 1)},
    }
    dom = max(kern, key=lambda k: kern[k]["ms"])
    ach = kern[dom]["GB/s"]
    # the towers against the bf16 MFMA peak: T1 = forward + backward-data of both towers
    # (2 x 2 x 2B x sum_l in_l * out_l flop), T2 = weight gradients (2 x 2B x sum_l in_l * out_l)
    towers = {}
    if step.towers is not None:
        macs = sum(i * o for i, o in zip([D] + layers[:-1], layers))
        t_t1 = time_kernel(lambda: step.towers.fwd_bwd(step.pooled, step.gpooled, step.params, step.labels,
                                                       step.logits), args.kernel_iters)
        t_t2 = time_kernel(lambda: step.towers.wgrad(step.loss), args.kernel_iters)
        for name, t_ms, fl in (("tower_fwd_bwd", t_t1, 8 * B * macs), ("tower_wgrad", t_t2, 4 * B * macs)):
            tf = fl / t_ms / 1e9
            towers[name] = {"ms": round(t_ms, 5), "flop": fl, "TFLOP/s": round(tf, 1),
                            "frac_of_bf16_peak": round(tf / MFMA_BF16_PEAK_TFS, 4)}
    roofline = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "bytes_per_launch": kern[dom]["bytes"],
                "kernels": kern, "lookups": nnz, "unique_rows": uniq, "towers_mfma": towers}
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_baseline(args, num_users, num_items, D, B, layers)
    return value, ms, loss, roofline, cpu, steps_run


def run_multi(args, world, rank, local_rank):
    import two_tower_recommender_model_amd as tt
    from two_tower_recommender_model_amd.task import TwoTower, TwoTowerTrainTask
    from two_tower_recommender_model_amd.torchrec.datasets.utils import Batch
    from two_tower_recommender_model_amd.torchrec.distributed.model_parallel import DistributedModelParallel
    from two_tower_recommender_model_amd.torchrec.modules.embedding_configs import EmbeddingBagConfig
    from two_tower_recommender_model_amd.torchrec.modules.embedding_modules import EmbeddingBagCollection
    from two_tower_recommender_model_amd.torchrec.optim.rowwise_adagrad import RowWiseAdagrad
    from two_tower_recommender_model_amd.torchrec.sparse.jagged_tensor import KeyedJaggedTensor
    from torch.distributed.optim import _apply_optimizer_in_backward

    num_users, num_items, D, B, layers = WORKLOADS[args.workload]
    dev = torch.device("cuda", local_rank)
    cfgs = [EmbeddingBagConfig(name="t_user_id", embedding_dim=D, num_embeddings=num_users, feature_names=["user_id"]),
            EmbeddingBagConfig(name="t_product_id", embedding_dim=D, num_embeddings=num_items,
                               feature_names=["product_id"])]
    ebc = EmbeddingBagCollection(tables=cfgs, device=torch.device("meta"))
    task = TwoTowerTrainTask(TwoTower(ebc, layers, device=dev))
    _apply_optimizer_in_backward(RowWiseAdagrad, task.two_tower.ebc.parameters(), {"lr": 0.01})
    model = DistributedModelParallel(module=task, device=dev)
    dense = [p for n, p in model.named_parameters() if "embedding_bags" not in n and p.numel() > 0]
    opt = torch.optim.Adam(dense, lr=0.01)
    from two_tower_recommender_model_amd import ops

    batches = []
    for cols, lab in synth_batches(num_users, num_items, B, 8, dev, args.ids, seed=1 + rank):
        v, l, o, _ = ops.kjt_build_mod_dropzero(cols, [num_users, num_items])
        n = int(o[-1])
        kjt = KeyedJaggedTensor(["user_id", "product_id"], v[:n], lengths=l, offsets=o, stride=B)
        batches.append(Batch(torch.zeros(1, device=dev), kjt, lab))

    def one(i):
        opt.zero_grad(set_to_none=True)
        loss, _ = model(batches[i % len(batches)])
        loss.backward()
        opt.step()
        return loss

    for i in range(args.warmup):
        one(i)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = one(i)
    torch.cuda.synchronize()
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], device=dev)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt)
    return world * args.steps * B / dt, dt / args.steps * 1e3, float(loss)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    num_users, num_items, D, B, layers = WORKLOADS[args.workload]
    config = {"workload": f"{args.workload}: {num_items // 1_000_000}M items x {num_users // 1_000_000}M users, "
                          f"emb_dim {D}, towers {layers}, single-hot {args.ids} ids",
              "global_batch": B * world, "per_gpu_batch": B, "emb_dim": D, "tower_dtype": "bf16 (MFMA, fp32 acc)",
              "parallelism": "single-gpu hipgraph" if world == 1 else f"rw-sharded tables + dp towers x{world}"}
    if world == 1:
        value, ms, loss, roofline, cpu, steps_run = run_single(args)
    else:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        value, ms, loss = run_multi(args, world, rank, local_rank)
        roofline, cpu, steps_run = None, None, args.steps
    if rank == 0:
        out = {"metric": "training pairs/sec at batch 8192 (per GPU)", "value": round(value, 1), "unit": "pairs/s",
               "n_gpus": world, "steps": steps_run, "warmup": args.warmup, "ms_per_step": round(ms, 5),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
               "data": "synthetic (uniform ids, Bernoulli labels), random-init weights", "config": config,
               "loss": loss, "roofline": roofline, "cpu_baseline": cpu}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
