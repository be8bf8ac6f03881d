#!/usr/bin/env python3
"""Benchmark: training pairs/s of the two-tower step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload northstar|config2]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (default = BASELINE.json north star): synthetic 100M-item x 50M-user two-tower, emb_dim
128, batch 8192 per GPU, towers [128, 64], single-hot ids uniform over each table (ids kept in HBM),
labels Bernoulli(0.5), random-init weights. One "step" = the full training step: device KJT build,
pooled forward, towers fwd (bf16 MFMA), dot + BCE, towers bwd, fused dedup + row-wise Adagrad on the
tables, Adam on the towers.

N = 1: the fused ring step replayed as HIP graphs. N > 1: one process per GPU over RCCL running the
pipelined sharded step (`sharded.FusedShardedTwoTowerStep`: table-wise at N = 2, row-wise from N = 4,
data-parallel towers, two fixed-size all-to-alls per step captured into the HIP graphs with the
kernels; config 5: `sharded_kjt.FusedShardedKJTStep`, three). `python bench.py --gpus N` without a
launcher starts `torch.distributed.run --nproc-per-node N` itself as a child process (before any GPU
call), relays its output and exits with its status; under a launcher the world size must equal
--gpus. Timing: W untimed steps, synchronize + barrier, K timed steps, synchronize (each rank's clock
read here) + barrier, max over ranks (the closing barrier's collective outside the interval, its
inclusive figure reported beside: end_timed_region); rank 0 prints ONE JSON line.
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

import numpy as np

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
    # SURVEY 8(d) config 5 on one GPU (both tables fit in 288 GB): multi-hot bags, lengths U{1..39}
    "config5": (50_000_000, 100_000_000, 128, 16384, [128, 64]),
}
MULTIHOT = {"config5": 39}  # workload -> max bag length (KJT input, bags of 1..max ids)
# sharded-only workloads: single-hot features, one table each, query features first;
# they run the sharded step at every N (at N = 1 over a one-rank group)
SIDE = 1_000_000
SHARDED = {
    # config 3: 8 table-wise features per tower (user_id 50M, product_id 100M, 14 side tables of 1M)
    "config3": dict(N=[50_000_000] + [SIDE] * 7 + [100_000_000] + [SIDE] * 7, Fq=8, D=128, B=8192,
                    layers=[128, 64], plan="tw", ids="uniform", seed=2),
    # config 4: a 1B-row item table row-wise over the ranks (125M rows each at N = 8), the 50M-row
    # user table table-wise (on the last rank), single-hot Zipf ids
    "config4": dict(N=[50_000_000, 1_000_000_000], Fq=1, D=128, B=8192, layers=[128, 64], plan="config4",
                    ids="zipf", seed=3),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="northstar", choices=sorted(WORKLOADS) + sorted(SHARDED))
    ap.add_argument("--ids", default=None, choices=["uniform", "zipf"],
                    help="id distribution (default uniform; config4: zipf)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=0,
                    help="table rows of the CPU sample (0: the workload's full tables when host RAM allows)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline: timed seconds of steps")
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--batches", type=int, default=64,
                    help="resident synthetic batches cycled by the single-hot bench (64 x 16,384 rows x 512 B "
                         "= 537 MB touched: past the 256 MiB Infinity Cache)")
    ap.add_argument("--kernel-iters", type=int, default=50)
    ap.add_argument("--steps-per-graph", type=int, default=None, choices=[1, 2, 4, 8, 16, 32],
                    help="steps per HIP graph (default 8)")
    ap.add_argument("--host-fed", action="store_true",
                    help="feed host batches through the 3-stage host pipeline (pinned staging, async H2D on a "
                         "copy stream, graph replay): the PCIe-inclusive rate, reported beside the resident one")
    ap.add_argument("--no-kjt-ahead", action="store_true",
                    help="multi-hot workloads: group each batch inside its own step instead of one step ahead")
    ap.add_argument("--sharded", action="store_true",
                    help="run the sharded (multi-GPU) step even at N = 1 (under torch.distributed.run)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "rccl", "peer"],
                    help="sharded steps (single-hot and config 5): auto (default) = device-initiated into "
                         "IPC-mapped peer buffers (sharded.PeerComm) when its startup self-test passes on every "
                         "rank, else RCCL; rccl = all_to_all_single; peer = PeerComm or fail")
    ap.add_argument("--overlap", action="store_true",
                    help="sharded step: T2 on a parallel graph branch beside exchange A (default: inside launch U, "
                         "one stream; the branch measured slower at world 1, DESIGN.md section 6)")
    ap.add_argument("--path", default="fused", choices=["fused", "dropin"],
                    help="dropin: the reference's own loop (DistributedModelParallel + TrainPipelineSparseDist."
                         "progress + KeyedOptimizerWrapper(Adam) + RowWiseAdagrad in backward, 03_model_training.py:"
                         "612-625, :770-829) on the torchrec shim, batches already device KJTs (the device KJT "
                         "builder in place of the host transform); progress() dispatches to the fused ring "
                         "(dropin.py). Also times the same loop with the dispatch off (the generic per-op path)")
    ap.add_argument("--plan", default="auto", choices=["auto", "tw", "rw"],
                    help="N > 1 sharding plan of the two tables: tw = table-wise (users on rank 0, items on rank "
                         "1), rw = row-wise over all ranks; auto = tw at N = 2 (the same per-rank load as rw), rw "
                         "from N = 4 (tw would leave N - 2 ranks without a table and give the two owners N / 2 x "
                         "the lookups of a row-wise owner; DESIGN.md section 6)")
    return ap.parse_args()


def synth_cols(Ns, B, n, device, ids, seed):
    """n batches of single-hot id columns (one per table of Ns) and Bernoulli(0.5) labels."""
    g = torch.Generator(device=device).manual_seed(seed)
    out = []

    def zipf(N):  # Zipf-like (s ~ 1.05) over randomly permuted ranks: heavy hot rows
        u01 = torch.rand(B, generator=g, device=device, dtype=torch.float64)
        r = torch.floor(torch.exp(u01 * torch.log(torch.tensor(float(N), device=device, dtype=torch.float64))))
        return (r.to(torch.int64) * 2654435761) % N

    for _ in range(n):
        if ids == "uniform":
            cols = [torch.randint(0, N, (B,), generator=g, device=device, dtype=torch.int64) for N in Ns]
        else:
            cols = [zipf(N) for N in Ns]
        lab = torch.randint(0, 2, (B,), generator=g, device=device, dtype=torch.int32)
        out.append((cols, lab))
    return out


def synth_batches(num_users, num_items, B, n, device, ids, seed):
    return synth_cols([num_users, num_items], B, n, device, ids, seed)


def tw_plan(Ns, W):
    """Table-wise owners: tables by size, largest first, each to the rank holding the fewest tables
    (every table brings the same B lookups per source), then the fewest bytes."""
    owners = [0] * len(Ns)
    cnt, byt = [0] * W, [0] * W
    for f in sorted(range(len(Ns)), key=lambda f: -Ns[f]):
        r = min(range(W), key=lambda r: (cnt[r], byt[r]))
        owners[f] = r
        cnt[r] += 1
        byt[r] += Ns[f]
    return owners


def sharded_spec(args, world):
    """(N list, Fq, D, B, layers, sharding, owners, ids, seed, plan description) of the sharded step."""
    if args.workload in SHARDED:
        sp = SHARDED[args.workload]
        N, Fq, D, B, layers = sp["N"], sp["Fq"], sp["D"], sp["B"], sp["layers"]
        ids = args.ids or sp["ids"]
        if sp["plan"] == "tw":
            owners = tw_plan(N, world)
            return (N, Fq, D, B, layers, ["table_wise"] * len(N), owners, ids, sp["seed"],
                    f"table-wise ({len(N)} tables over {world} ranks, greedy by table count then bytes: {owners})")
        # config4: items row-wise, users table-wise on the last rank
        per_rank = (N[1] // world + N[0] * (world == 1)) * (4 * D + 4)
        if per_rank > 200 << 30:
            raise SystemExit(f"config4 needs at least 4 GPUs (the 1B-row table is {N[1] * 4 * D / 2**30:.0f} GiB; "
                             f"{per_rank / 2**30:.0f} GiB per rank at N = {world})")
        return (N, Fq, D, B, layers, ["table_wise", "row_wise"], [world - 1, 0], ids, sp["seed"],
                f"product_id row-wise (blocks of ceil(N / {world}) rows), user_id table-wise on rank {world - 1}")
    num_users, num_items, D, B, layers = WORKLOADS[args.workload]
    N = [num_users, num_items]
    plan = args.plan if args.plan != "auto" else ("tw" if world == 2 else "rw")
    if plan == "tw" and world < 2:
        plan = "rw"  # one rank holds everything either way
    if plan == "tw":
        return (N, 1, D, B, layers, ["table_wise"] * 2, [0, 1], args.ids or "uniform", 1,
                "table-wise (user_id -> rank 0, product_id -> rank 1)")
    return (N, 1, D, B, layers, ["row_wise"] * 2, [0, 0], args.ids or "uniform", 1,
            f"row-wise (blocks of ceil(N / {world}) rows)")


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


def cpu_threads() -> int:
    """Host threads of the CPU baseline: every core this process may run on, capped by the CPU share
    the host grants one GPU (the box exports OMP_NUM_THREADS = its per-GPU share; nproc there shows
    the whole machine)."""
    n = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(share))) if share and share.isdigit() else n


def cpu_tables(rows, D, threads, seed=0):
    """The oracle's tables at the requested rows, filled U(-sqrt(1/N), sqrt(1/N)) (torchrec EBC init)
    in parallel chunks (torch's CPU uniform_ runs on one thread: ~1.5 s/GB)."""
    import concurrent.futures as cf

    out = []
    for t, n in enumerate(rows):
        w = torch.empty(n, D)
        a = (1.0 / n) ** 0.5
        step = max(1, -(-n // (4 * threads)))

        def fill(i, w=w, a=a, t=t):
            w[i:i + step].uniform_(-a, a, generator=torch.Generator().manual_seed(seed * 7919 + t * 104729 + i))

        with cf.ThreadPoolExecutor(threads) as ex:
            list(ex.map(fill, range(0, n, step)))
        out.append(w)
    return out


def cpu_rows(args, num_users, num_items, D):
    """Full tables when this host can hold them, else scaled-down tables
    (--cpu-rows, default 2M rows each when RAM is short). Returns (rows, description)."""
    full = (num_users + num_items) * (4 * D + 4)
    try:
        import psutil

        avail = psutil.virtual_memory().available
    except Exception:  # noqa: BLE001
        avail = 0
    if args.cpu_rows == 0 and avail > 1.5 * full + (8 << 30):
        return (num_users, num_items), "full tables"
    n = args.cpu_rows or 2_000_000
    rows = (min(n, num_users), min(n, num_items))
    if args.cpu_rows:
        return rows, "tables scaled down (--cpu-rows)"
    return rows, (f"tables scaled down (host RAM available {avail / 2**30:.0f} GiB < 1.5 x "
                  f"{full / 2**30:.0f} GiB + 8 GiB)")


def cpu_baseline(args, num_users, num_items, D, B, layers):
    """The oracle (CPU restatement of TorchRec's unsharded CPU path, sparse touched-row update) on
    this host's cores, bounded sample: full B, D, towers, full tables when RAM allows; steps until
    --cpu-seconds of CPU work (at least --cpu-steps); value = B / median step time."""
    from oracle import ref

    threads = cpu_threads()
    torch.set_num_threads(threads)
    rows, how = cpu_rows(args, num_users, num_items, D)
    st = ref.init_state([1, 1], [D, D], [0, 1], [0], [1], layers, seed=0)
    st.tables = cpu_tables(rows, D, threads)
    st.states = [torch.zeros(n) for n in rows]
    g = torch.Generator().manual_seed(0)
    batches = []
    for _ in range(4):
        cols = [torch.randint(0, rows[0], (B,), generator=g), torch.randint(0, rows[1], (B,), generator=g)]
        lab = torch.randint(0, 2, (B,), generator=g)
        v, l, o = ref.kjt_build([c.numpy() for c in cols], list(rows))
        batches.append((torch.from_numpy(v), torch.from_numpy(o), lab))
    for i in range(10):  # 10 warm-up steps, then the median of the timed ones
        v, o, lab = batches[i % 4]
        ref.train_step(st, v, o, B, lab, 0.01, 0.01)
    t0 = time.perf_counter()
    times = []
    while len(times) < args.cpu_steps or time.perf_counter() - t0 < args.cpu_seconds:
        v, o, lab = batches[len(times) % 4]
        t = time.perf_counter()
        ref.train_step(st, v, o, B, lab, 0.01, 0.01)
        times.append(time.perf_counter() - t)
    dt = time.perf_counter() - t0
    q10, q50, q90 = np.percentile(times, [10, 50, 90])
    return {
        "value": round(float(B / q50), 1), "unit": "pairs/s", "cores": threads, "kind": "port",
        "sample": f"median of {len(times)} timed steps ({dt:.1f} s, after 10 warm-up) of the oracle train_step "
                  f"(torch CPU fp32: embedding_bag sum, towers {layers}, BCE, sparse row-wise Adagrad, Adam) at "
                  f"B={B}, D={D}, {how} ({rows[0]}x{D} / {rows[1]}x{D}); step p10/p50/p90 "
                  f"{q10 * 1e3:.2f}/{q50 * 1e3:.2f}/{q90 * 1e3:.2f} ms; {threads} threads of "
                  f"{len(os.sched_getaffinity(0))} in the affinity mask; host CPU {cpu_model()}",
    }


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def lookup_stats(step, batches):
    """Kept lookups, unique (table, row) pairs and rows looked up exactly once per step, averaged
    over the resident batches."""
    nnz = uniq = once = 0
    for cols, _ in batches:
        keys = torch.cat([(c % n) + (t << 40) for t, (c, n) in enumerate(zip(cols, step.num_embeddings))])
        nz = torch.cat([c != 0 for c in cols])
        nnz += int(nz.sum())
        u, cnt = torch.unique(keys[nz], return_counts=True)
        uniq += int(u.numel())
        once += int((cnt == 1).sum())
    n = len(batches)
    return nnz // n, uniq // n, once // n


def launch_bytes(step, nnz: int, uniq: int, once: int):
    """Per launch of the production ring step: ``alg`` = the launch's share of
    the SURVEY.md 8(d) algorithmic bytes (the FBGEMM convention: every lookup's id + row in the
    forward, 4 B length + 4D pooled write + 4D gradient read per bag, unique rows' weight + state
    read and write in the backward); ``design`` = what the launch moves by design (incl. the T1 -> T2
    bf16 operand strips, the split-K slabs and the dedup slots); ``flop`` = tower MFMA flops.
      t1 = gather + towers fwd/bwd + the in-place update of the `once` rows looked up once: 8(d) ids
           fwd + rows + lengths + pooled (kept on chip) and, for those rows, ids bwd + gradient
           (on chip) + weight and state read-modify-write;
      t2 = tower weight gradients + Adam scalars + the next batch's dedup insert: no 8(d) bytes;
      k3 = resolver + update of the rows looked up more than once + T3: the rest of 8(d)."""
    D, B, F = step.dims[0], step.B, step.F
    L = step.layer_sizes
    idb = 8 if step.id_dtype == torch.int64 else 4
    macs = sum(i * o for i, o in zip([D] + L[:-1], L))
    opnd = 2 * B * 2 * (D + L[0] + (L[0] + L[1]))  # bf16 X^T, act^T, dZ^T of both towers (T1 -> T2)
    P = step.params.numel()
    cdiv = lambda a, b: -(-a // b)  # noqa: E731
    S = min(64, cdiv(B, 256))  # staged T2 slices of whole 256-row passes (tower.hip tower_layout)
    S = cdiv(B, cdiv(cdiv(B, S), 256) * 256)
    multi = nnz - once  # lookups of rows looked up more than once
    t1_design = (F * B * idb + B * 4 + nnz * 4 * D + F * B * 12 + once * (8 * D + 8) + multi * 4 * D + opnd)
    t2_design = opnd + S * P * 4 + F * B * (idb + 20)
    k3_design = (F * B * (4 + 64) + (uniq - once) * (8 * D + 8) + multi * 4 * D + S * P * 4 + 6 * P * 4 + 4 * P)
    t1_alg = nnz * (8 + 4 * D) + F * B * (4 + 4 * D) + once * (8 + 4 * D + 8 * D + 8)
    k3_alg = multi * 8 + (F * B - once) * 4 * D + (uniq - once) * (8 * D + 8)
    rows_t1 = uses_rows_t1(step)
    out = {"t1": {"alg_bytes": t1_alg, "design_bytes": t1_design, "flop": 8 * B * macs,
                   "what": ("tower_rows_kernel<UPD> (row-owned waves, whole chain in registers)" if rows_t1 else
                            "tower_l2_kernel<UPD>") + ": EBC gather + both towers fwd/bwd + row-wise Adagrad of the rows "
                           "looked up once"},
            "t2": {"alg_bytes": 0, "design_bytes": t2_design, "flop": 4 * B * macs,
                   "what": "tower_wgrad_insert_kernel: tower weight gradients + Adam scalars + next batch's dedup insert"},
            "k3": {"alg_bytes": k3_alg, "design_bytes": k3_design, "flop": 0,
                   "what": "tower_update_dedup_resolve_kernel: next batch's deferred inserts + row-wise Adagrad of the "
                           "rows looked up more than once + slab reduction + Adam + bf16 copies"},
            "_emb_path_bytes": t1_alg + k3_alg}
    if getattr(step, "ring_tail", False):  # T2 + insert + row update, then T3
        t3_design = S * P * 4 + 6 * P * 4 + 4 * P
        out["tail"] = {"alg_bytes": k3_alg, "design_bytes": t2_design + k3_design - t3_design, "flop": 4 * B * macs,
                       "what": "tower_tail_kernel: tower weight gradients + next batch's complete dedup insert + "
                               "row-wise Adagrad of the rows looked up more than once"}
        out["t3"] = {"alg_bytes": 0, "design_bytes": t3_design, "flop": 0,
                     "what": "tower_update_kernel: slab reduction + Adam + bf16 weight copies"}
        del out["t2"], out["k3"]
    return out


def pmc_traffic(kernel_name: str, workload: str = "northstar"):
    """HBM bytes per launch of `kernel_name` from the newest committed PMC summary of this workload
    (profiles/*pmc*.json; a non-default workload's summaries carry its name, e.g.
    r01_pmc_traffic_config5.json; FETCH_SIZE/WRITE_SIZE passes of scripts/pmc_traffic.sh,
    gfx950-corrected), or None."""
    import glob
    files = glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))
    others = [w for w in WORKLOADS if w != "northstar"] + ["zipf"]
    if workload == "northstar":
        files = [f for f in files if not any(w in os.path.basename(f) for w in others)]
    else:
        files = [f for f in files if workload in os.path.basename(f)]
    files = sorted(files, key=os.path.basename)
    for fn in reversed(files):  # newest summary that holds the kernel
        with open(fn) as f:
            d = json.load(f)
        # several instantiations may match (the ring's first step runs T1 without the in-place
        # update once): the steady-state one is the one launched most often
        hits = [v for k, v in d.get("kernels", {}).items() if kernel_name in k]
        if hits:
            v = max(hits, key=lambda e: max(e.get("launches") or [0]))
            return v.get("hbm_bytes"), os.path.relpath(fn, ROOT)
    return None, None


KERNEL_NAMES = {"t1": "tower_l2_kernel", "t2": "tower_wgrad_insert_kernel", "k3": "tower_update_dedup_resolve_kernel",
                "tail": "tower_tail_kernel", "t3": "tower_update_kernel"}


def uses_rows_t1(step) -> bool:
    """The fused gather T1 of the [128, 64] towers over 128- or 64-wide rows is the row-owned kernel
    (tower.hip launch_t1: tower_rows_kernel)."""
    return bool(getattr(step, "gather", False)) and step.layer_sizes == [128, 64] and \
        getattr(step, "in_q", 0) == getattr(step, "in_c", 0) and getattr(step, "in_q", 0) in (64, 128)


def kernel_names(step) -> dict:
    names = dict(KERNEL_NAMES)
    if uses_rows_t1(step):
        names["t1"] = "tower_rows_kernel"
    return names


def synth_kjt_batches(num_users, num_items, B, maxlen, n, device, ids, seed):
    """Multi-hot KJT batches (keys user, item; key-major bags of Uniform{1..maxlen} ids in range)."""
    g = torch.Generator(device=device).manual_seed(seed)
    out = []
    for _ in range(n):
        lengths = torch.randint(1, maxlen + 1, (2 * B,), generator=g, device=device, dtype=torch.int32)
        offsets = torch.zeros(2 * B + 1, dtype=torch.int32, device=device)
        offsets[1:] = torch.cumsum(lengths, 0)
        vals = []
        for f, N in enumerate((num_users, num_items)):
            k = int(lengths[f * B:(f + 1) * B].sum())
            if ids == "uniform":
                vals.append(torch.randint(0, N, (k,), generator=g, device=device, dtype=torch.int64))
            else:
                u01 = torch.rand(k, generator=g, device=device, dtype=torch.float64)
                r = torch.floor(torch.exp(u01 * torch.log(torch.tensor(float(N), device=device, dtype=torch.float64))))
                vals.append((r.to(torch.int64) * 2654435761) % N)
        lab = torch.randint(0, 2, (B,), generator=g, device=device, dtype=torch.int32)
        out.append((torch.cat(vals), offsets, lab))
    return out


def end_timed_region(t0: float, dev) -> tuple:
    """Close a multi-rank timed region: this rank's clock is read right after its device
    synchronize, then the closing barrier runs, then the MAX over ranks. Every rank started its
    clock on leaving the same opening barrier, so max(end - t0) is when the last rank's steps were
    done; the closing barrier's own collective (35-60 us over RCCL even at world 1,
    profiles/r06sh_barrier.log) is not the job's work. Returns (seconds, seconds with the closing
    barrier), both max over ranks; the second is reported beside the line."""
    t1 = time.perf_counter()
    dist.barrier()
    t2 = time.perf_counter()
    dt = torch.tensor([t1 - t0, t2 - t0], device=dev, dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    return float(dt[0]), float(dt[1])


def run_multihot(args):
    """SURVEY 8(d) config 5 shape at N = 1: the fused step on multi-hot KJT input (tt_pooled_fwd ->
    fused towers T1 -> tiled tt_bwd_prepare (side stream) -> T2/T3 (side stream) ->
    tt_bwd_rowwise_adagrad), one HIP graph per resident batch."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    num_users, num_items, D, B, layers = WORKLOADS[args.workload]
    maxlen = MULTIHOT[args.workload]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    ahead = not args.no_kjt_ahead
    k = (args.steps_per_graph or 8) if ahead else 1  # several steps per graph: no gap between them
    batches = synth_kjt_batches(num_users, num_items, B, maxlen, max(4, k), dev, args.ids, seed=4)
    cap = max(v.numel() for v, _, _ in batches)
    step = FusedTwoTowerStep([num_users, num_items], [D, D], [0], [1], layers, B, dev, lr_emb=0.01, lr_dense=0.01,
                             id_dtype=torch.int64, seed=0, max_lookups=cap)
    # pipelined grouping: batch i+1's tt_bwd_prepare runs on the side stream during step i
    step.capture_pool_kjt(batches, ahead=ahead, steps_per_graph=k)

    def run(n):
        step.replay_pool(n)

    # the timed steps grouped into k-step graphs (the remainder first, in aligned smaller graphs):
    # a graph ends by joining its last step's side branches, so each graph launch costs the stream
    # an idle gap; regrouped BEFORE the warm-up, which runs right up to the timed region
    step.align_pool(args.steps, after=args.warmup)
    run(args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms = dt / args.steps * 1e3
    value = args.steps * B / dt
    loss = float(step.loss)
    # per-launch device time: eager steps with HIP events around each launch on its stream
    step._timing = []
    try:
        for i in range(min(args.steps, 20)):
            step._timing.append({})
            step.pool_step_eager()
        torch.cuda.synchronize()
        acc = {}
        for mk in step._timing:
            for name, (a, b) in mk.items():
                acc.setdefault(name, []).append(a.elapsed_time(b))
    finally:
        step._timing = None
    timed = {k: sum(v) / len(v) for k, v in acc.items()}
    nnz = sum(v.numel() for v, _, _ in batches) // len(batches)
    uniq = 0
    for v, o, _ in batches:
        nb = int(o[B])
        uniq += int(torch.unique(torch.cat([v[:nb], v[nb:] + (1 << 40)])).numel())
    uniq //= len(batches)
    FB = 2 * B
    # alg = SURVEY 8(d) bytes (ids + rows per lookup in the forward, ids again in the backward, 4 B
    # length + 4D pooled write + 4D gradient read per bag, unique rows' weight + state read and write);
    # design = what the launches move (the update reads a gradient row per lookup, mostly cache hits)
    kern = {
        "fwd": {"alg_bytes": nnz * (8 + 4 * D) + FB * (4 + 4 * D), "design_bytes": nnz * (8 + 4 * D) + FB * (4 + 4 * D),
                "kernel": "pooled_fwd_kernel",
                "what": "tt_pooled_fwd: segmented gather + sum pool (8 B id + 4D row per lookup, 4D per bag)"},
        "prep": {"alg_bytes": nnz * 8, "design_bytes": nnz * (8 + 4 + 4) + FB * 4,
                 "kernel": "bwd_tile_hash + scan + bwd_tile_scatter",
                 "what": "tt_bwd_prepare: ids read, per-lookup entry word, segment scatter"},
        "upd": {"alg_bytes": FB * 4 * D + uniq * (8 * D + 8), "design_bytes": nnz * (4 * D + 4) + uniq * (8 * D + 8),
                "kernel": "bwd_adagrad_direct_kernel (+ narrow and hot-row launches)",
                "what": "tt_bwd_rowwise_adagrad: weight row + state read+write per unique row (8(d)), gradient row "
                        "per bag (8(d)); by design a gradient row per lookup (once-looked-up rows in lookup order)"},
        "t1": {"alg_bytes": None, "kernel": "tower_fwd_bwd_kernel", "what": "fused towers fwd/bwd + dot/BCE"},
        "t2t3": {"alg_bytes": None, "kernel": "tower_wgrad + tower_update", "what": "tower weight grads + Adam (side stream)"},
    }
    pool_in_t1 = "fwd" not in timed  # tt_tower_fwd_bwd_kjt: the sum pool runs inside T1
    if pool_in_t1:
        kern["t1"].update(alg_bytes=kern["fwd"]["alg_bytes"], design_bytes=kern["fwd"]["design_bytes"],
                          kernel="tower_l2_kernel",
                          what="tt_tower_fwd_bwd_kjt: the segmented gather + sum pool of every bag (8 B id + 4D row "
                               "per lookup, 4D per bag) inside the fused towers fwd/bwd + dot/BCE")
        del kern["fwd"]
    for name, k in kern.items():
        if name in timed:
            k["ms"] = round(timed[name], 5)
            if k["alg_bytes"]:
                k["alg_GB/s"] = round(k["alg_bytes"] / timed[name] / 1e6, 1)
                k["design_GB/s"] = round(k["design_bytes"] / timed[name] / 1e6, 1)
    emb_bytes = nnz * (16 + 4 * D) + FB * (4 + 8 * D) + uniq * (8 * D + 8)
    fwd_name = "t1" if pool_in_t1 else "fwd"
    emb_ms = sum(timed.get(n, 0.0) for n in (fwd_name, "prep", "upd"))
    dom = max((fwd_name, "upd"), key=lambda n: timed.get(n, 0.0))
    traffic, src = pmc_traffic(kern[dom]["kernel"].split()[0],
                               args.workload if args.ids == "uniform" else f"{args.workload}_{args.ids}")
    ach = kern[dom].get("alg_GB/s")
    roofline = {"bound": "hbm", "kernel": kern[dom]["kernel"], "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None, "traffic": traffic, "traffic_source": src,
                "alg_bytes_per_launch": kern[dom]["alg_bytes"], "design_bytes_per_launch": kern[dom]["design_bytes"],
                "ms_per_launch": kern[dom].get("ms"),
                "timing": "HIP events around each launch on its stream over eager steps of the same sequence",
                "kernels": kern, "lookups": nnz, "unique_rows": uniq,
                "embedding_path": {"bytes_per_step": emb_bytes, "ms": round(emb_ms, 5),
                                   "GB/s": round(emb_bytes / emb_ms / 1e6, 1) if emb_ms else None,
                                   "frac": round(emb_bytes / emb_ms / 1e6 / HBM_PEAK_GBS, 4) if emb_ms else None,
                                   "GB/s_over_step": round(emb_bytes / ms / 1e6, 1),
                                   "frac_over_step": round(emb_bytes / ms / 1e6 / HBM_PEAK_GBS, 4),
                                   "note": "SURVEY 8(d) bytes over the summed time of the three embedding "
                                           "launches (fwd — T1 when the sum pool runs inside it, prepare, fused "
                                           "Adagrad), and over the step"}}
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_baseline_multihot(args, num_users, num_items, D, B, layers, maxlen)
    return value, ms, loss, roofline, cpu, args.steps


def run_multi_kjt(args, world, rank, local_rank):
    """Config 5 over W ranks (or one rank with --sharded): the capturable multi-hot sharded step
    (sharded_kjt.FusedShardedKJTStep: users table-wise on the last rank, items row-wise over all
    ranks; three fixed-size all-to-alls per step, ids in, pooled rows out, bag gradients back, over
    RCCL), one HIP graph per resident batch (eager under TT_REHEARSE_GLOO). B = 16,384 bags per
    feature and rank, bags of Uniform{1..39} ids. Capacity: the most ids any rank's resident batch
    sends to one destination (all-reduced)."""
    from two_tower_recommender_model_amd.sharded import PeerComm, exchange_comm
    from two_tower_recommender_model_amd.sharded_kjt import FusedShardedKJTStep, route_counts

    num_users, num_items, D, B, layers = WORKLOADS[args.workload]
    maxlen = MULTIHOT[args.workload]
    N = [num_users, num_items]
    sharding, owners = ["table_wise", "row_wise"], [world - 1, 0]
    dev = torch.device("cuda", local_rank % torch.cuda.device_count())
    comm, xdesc = exchange_comm(args.exchange, device=dev)
    peer = isinstance(comm, PeerComm)
    batches = synth_kjt_batches(num_users, num_items, B, maxlen, 4, dev, args.ids, seed=4 * 1000 + 1 + rank)
    need = torch.zeros(1, dtype=torch.int64)
    for v, o, _ in batches:
        need = torch.maximum(need, route_counts(v, o, B, N, sharding, owners, world).max().reshape(1))
    need = need.to(dev)
    dist.all_reduce(need, op=dist.ReduceOp.MAX)
    cap = -(-int(need) // 8) * 8
    step = FusedShardedKJTStep(comm, N, D, layers, B, dev, cap=cap, sharding=sharding, tw_owners=owners,
                               lr_emb=0.01, lr_dense=0.01, seed=0)
    graphs = os.environ.get("TT_REHEARSE_GLOO") != "1" or peer
    if graphs:
        step.capture_pool(batches)
        run = step.run
    else:
        step.warmup()
        state = {"i": 0}

        def run(n):
            step.run_eager(batches, n, state["i"])
            state["i"] += n

    run(args.warmup)
    torch.cuda.synchronize()
    step.check()
    dist.barrier()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    dt, dt_barrier = end_timed_region(t0, dev)
    step.check()
    loss = float(step.loss)
    step.release_graphs()
    if peer:
        dist.barrier()  # no rank unmaps a peer's buffer while that peer may still store into it
        comm.close()
    # SURVEY 8(d) embedding-path bytes per rank and step over the whole step (lookups of this rank's
    # batch, unique rows counted on it): nnz (8 id fwd + 8 id bwd + 4D row) + F B (4 + 8D) + U (8D + 8)
    nnz = sum(v.numel() for v, _, _ in batches) // len(batches)
    uniq = 0
    for v, o, _ in batches:
        nb = int(o[B])
        uniq += int(torch.unique(torch.cat([v[:nb], v[nb:] + (1 << 40)])).numel())
    uniq //= len(batches)
    emb_bytes = nnz * (16 + 4 * D) + 2 * B * (4 + 8 * D) + uniq * (8 * D + 8)
    ach = emb_bytes / (dt / args.steps) / 1e9
    roofline = {"bound": "hbm", "kernel": "whole sharded step (per rank)", "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "alg_bytes_per_step": emb_bytes, "lookups": nnz, "unique_rows": uniq,
                "timing": "SURVEY 8(d) bytes per rank over the max-over-ranks step time (collectives included)"}
    info = {"plan": f"users table-wise (rank {world - 1}) + items row-wise", "ids": args.ids, "capacity": cap,
            "exchange_bytes_per_rank": {"A_ids": 4 * step.sendA.numel(), "B_pooled": 4 * step.sendB.numel(),
                                        "C_grads": 4 * step.sendC.numel()},
            "collectives_per_step": 3, "mode": "hipgraph" if graphs else "eager", "exchange": xdesc,
            "ms_per_step_with_closing_barrier": round(dt_barrier / args.steps * 1e3, 5)}
    return world * args.steps * B / dt, dt / args.steps * 1e3, loss, info, roofline


def cpu_baseline_multihot(args, num_users, num_items, D, B, layers, maxlen):
    """The oracle train_step on multi-hot bags of the same shape (full tables when RAM allows)."""
    from oracle import ref

    threads = cpu_threads()
    torch.set_num_threads(threads)
    rows, how = cpu_rows(args, num_users, num_items, D)
    st = ref.init_state([1, 1], [D, D], [0, 1], [0], [1], layers, seed=0)
    st.tables = cpu_tables(rows, D, threads)
    st.states = [torch.zeros(n) for n in rows]
    bs = synth_kjt_batches(rows[0], rows[1], B, maxlen, 2, torch.device("cpu"), "uniform", seed=0)
    for i in range(4):
        ref.train_step(st, bs[i % 2][0], bs[i % 2][1], B, bs[i % 2][2], 0.01, 0.01)
    t0 = time.perf_counter()
    times = []
    while len(times) < args.cpu_steps or time.perf_counter() - t0 < args.cpu_seconds:
        v, o, lab = bs[len(times) % 2]
        t = time.perf_counter()
        ref.train_step(st, v, o, B, lab, 0.01, 0.01)
        times.append(time.perf_counter() - t)
    dt = time.perf_counter() - t0
    q10, q50, q90 = np.percentile(times, [10, 50, 90])
    return {"value": round(float(B / q50), 1), "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"median of {len(times)} timed steps ({dt:.1f} s, after 4 warm-up) of the oracle train_step on "
                      f"multi-hot bags (lengths U{{1..{maxlen}}}) at B={B}, D={D}, towers {layers}, {how} "
                      f"({rows[0]}x{D} / {rows[1]}x{D}); step p10/p50/p90 {q10 * 1e3:.1f}/{q50 * 1e3:.1f}/"
                      f"{q90 * 1e3:.1f} ms; {threads} threads; host CPU {cpu_model()}"}


def roofline_report(kern, timed, nnz, uniq, step, B, ms_step, workload="northstar", once=None):
    """``roofline`` of the dominant launch (T1): achieved = its SURVEY 8(d) bytes / its average
    device time; ``traffic`` = its HBM bytes per launch from the committed PMC summary; per-launch
    design bytes, flops and MFMA fractions beside it; the whole embedding path (8(d) bytes per step)
    over the step time and over the time of the two launches that carry it."""
    emb_path_bytes = kern.pop("_emb_path_bytes")
    names = kernel_names(step)
    out = {}
    for name, k in kern.items():
        ms = timed.get(name) if timed else None
        e = dict(k)
        e["kernel"] = names[name]
        if ms:
            e["ms"] = round(ms, 5)
            e["alg_GB/s"] = round(k["alg_bytes"] / ms / 1e6, 1)
            e["design_GB/s"] = round(k["design_bytes"] / ms / 1e6, 1)
            if k["flop"]:
                e["TFLOP/s"] = round(k["flop"] / ms / 1e9, 1)
                e["frac_of_bf16_peak"] = round(k["flop"] / ms / 1e9 / MFMA_BF16_PEAK_TFS, 4)
        t, src = pmc_traffic(names[name], workload)
        e["pmc_hbm_bytes"], e["pmc_source"] = t, src
        out[name] = e
    path = {"bytes_per_step": emb_path_bytes,
            "GB/s_over_step": round(emb_path_bytes / ms_step / 1e6, 1),
            "frac_over_step": round(emb_path_bytes / ms_step / 1e6 / HBM_PEAK_GBS, 4)}
    if not timed:
        return {"bound": "hbm", "kernel": None, "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                "traffic": None, "kernels": out, "lookups": nnz, "unique_rows": uniq, "rows_looked_up_once": once, "embedding_path": path}
    dom = "t1"  # the longest launch, and the one that carries the forward's row reads
    emb_ms = timed.get("t1", 0.0) + timed.get("k3", timed.get("tail", 0.0))
    ach = out[dom]["alg_GB/s"]
    path.update({"ms_t1_k3": round(emb_ms, 5), "GB/s_over_t1_k3": round(emb_path_bytes / emb_ms / 1e6, 1),
                 "frac_over_t1_k3": round(emb_path_bytes / emb_ms / 1e6 / HBM_PEAK_GBS, 4),
                 "note": "SURVEY 8(d) bytes per step: over the whole step, and over T1 + K3 or the tail launch (the launches that "
                         "carry the embedding work; both also run tower work)"})
    return {"bound": "hbm", "kernel": names[dom], "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": out[dom]["pmc_hbm_bytes"],
            "traffic_source": out[dom]["pmc_source"], "alg_bytes_per_launch": out[dom]["alg_bytes"],
            "alg_bytes_rule": "SURVEY 8(d) share of T1: per kept lookup 8 B id + 4D row; per bag 4 B length + 4D "
                              "pooled row (kept on chip); per row looked up once 8 B id + 4D gradient (on chip) + "
                              "8D weight read/write + 8 B state read/write",
            "design_bytes_per_launch": out[dom]["design_bytes"], "ms_per_launch": out[dom]["ms"],
            "kernels": out, "lookups": nnz, "unique_rows": uniq, "rows_looked_up_once": once, "embedding_path": path}


def run_single(args):
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    num_users, num_items, D, B, layers = WORKLOADS[args.workload]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    step = FusedTwoTowerStep([num_users, num_items], [D, D], [0], [1], layers, B, dev, lr_emb=0.01,
                             lr_dense=0.01, id_dtype=torch.int64, seed=0)
    # 8 steps per graph by default: 32 measured 35.0 against 35.5-35.7 us/step in 96-step runs and
    # 35.9 against 36.5 at the default 50, but no better at 20 steps (37.40 / 37.38 us, 38.35 / 38.06
    # after 3 warm-up steps; profiles/r03_ring_steps_per_graph_ab*.log)
    spg = args.steps_per_graph or 8
    nb = max(spg, args.batches // spg * spg)
    batches = synth_batches(num_users, num_items, B, nb, dev, args.ids, seed=1)
    # the production ring: HIP graphs of k full steps over the resident batches (no input copies;
    # each step files the next batch's dedup table): a graph launch costs the host ~35-55 us, more
    # than a step's GPU time, so k > 1 keeps the GPU fed (single-step graphs for a remainder)
    k = spg
    step.capture_ring(batches, steps_per_graph=k)

    def run(n):
        step.run(n)

    # group the timed steps into graph launches (the remainder in aligned smaller graphs first, then
    # k-step graphs): a warmup or step count that is not a multiple of k would otherwise leave
    # single-step graphs in the timed region. Regrouped BEFORE the warmup, so the warmup's steps
    # run right up to the timed region (no capture pause between them)
    step.align_ring(args.steps, after=args.warmup)
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
    # ---- per-launch device time inside the replayed graphs: the same graphs re-captured with
    # event-record nodes around every kernel node (graph_timing.py), replayed for K steps;
    # eager steps with HIP events around each launch if the graph cannot be instrumented
    nnz, uniq, once = lookup_stats(step, batches)
    kern = launch_bytes(step, nnz, uniq, once)
    timed, timing_how = None, None
    if step.ring_supported():
        try:
            from two_tower_recommender_model_amd.graph_timing import GraphLaunchTimer

            step.capture_ring(batches, steps_per_graph=k, keep_graph=True)
            names = ["t1", "tail", "t3"] if step.ring_tail else ["t1", "t2", "k3"]
            nl = len(names)
            timers = [GraphLaunchTimer(g, list(range(nl * k))) for g in step.ring_graphs]
            acc = {n: [] for n in names}
            n_done, j = 0, 0
            while n_done < args.steps:
                step.ring_graphs[j % len(step.ring_graphs)].replay()
                torch.cuda.synchronize()
                for i, t_ms in enumerate(timers[j % len(timers)].elapsed()):
                    acc[names[i % nl]].append(t_ms)
                n_done, j = n_done + k, j + 1
            timed = {n: sum(v) / len(v) for n, v in acc.items()}
            timing_how = "HIP event-record nodes around each kernel node of the replayed step graphs (K steps)"
            for t in timers:
                t.close()
        except Exception as e:  # noqa: BLE001
            print(f"graph instrumentation unavailable ({e}); eager per-launch events", file=sys.stderr)
    if timed is None:
        timed = step.timed_ring(args.steps) if step.ring_supported() else step.timed_steps(batches, args.steps)
        timing_how = "HIP events around each launch on its stream over K eager steps of the same sequence"
    # an event-record node in front of a kernel node adds its own dispatch latency to the measured
    # span (about 2 us a launch on this stack); the spans are scaled so that they sum to the step
    # time measured without event nodes (the un-instrumented replay above), which puts each launch
    # within a few percent of rocprofv3's kernel-trace duration
    raw = dict(timed)
    tot = sum(raw.values())
    if timing_how and timing_how.startswith("HIP event-record nodes") and tot > ms:
        timed = {n: v * ms / tot for n, v in raw.items()}
        timing_how += ("; each span scaled by (step time without event nodes) / (sum of the spans) = "
                       f"{ms / tot:.3f}")
    roofline = roofline_report(kern, timed, nnz, uniq, step, B, ms,
                               args.workload if args.ids == "uniform" else f"{args.workload}_{args.ids}", once)
    roofline["timing"] = timing_how
    roofline["event_span_ms"] = {n: round(v, 5) for n, v in raw.items()}
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_baseline(args, num_users, num_items, D, B, layers)
    return value, ms, loss, roofline, cpu, steps_run


def run_dropin(args, world=1, rank=0, local_rank=0):
    """The reference's loop through the torchrec shim: main()'s wiring (EBC on meta, TwoTower,
    TwoTowerTrainTask, in-backward RowWiseAdagrad, DistributedModelParallel, KeyedOptimizerWrapper(Adam),
    TrainPipelineSparseDist; 03_model_training.py:770-829) and train()'s ``pipeline.progress`` loop
    (:612-625) over resident device KJT batches built by the device KJT builder (tt_kjt_build_mod_dropzero,
    the reference's transform_to_torchrec_batch semantics). progress() dispatches to the fused ring
    (dropin.py); K timed progress calls. Then the same model with the dispatch off (a fresh pipeline,
    TT_DROPIN_FUSED=0: the generic per-op path on the same storage) for a few steps.
    At world > 1 (the process group already initialised by main): DMP shards the tables by the
    default plan over the W ranks, progress() dispatches to the pipelined fused sharded step
    (dropin.FusedShardedDropin), every rank times its loop between barriers and the max is taken."""
    import itertools

    import two_tower_recommender_model_amd as tt
    from two_tower_recommender_model_amd import ops

    tt.install_torchrec_alias()
    from torch.distributed.optim import _apply_optimizer_in_backward
    from torchrec.datasets.utils import Batch
    from torchrec.distributed import TrainPipelineSparseDist
    from torchrec.distributed.model_parallel import DistributedModelParallel
    from torchrec.modules.embedding_configs import EmbeddingBagConfig
    from torchrec.modules.embedding_modules import EmbeddingBagCollection
    from torchrec.optim.keyed import KeyedOptimizerWrapper
    from torchrec.optim.rowwise_adagrad import RowWiseAdagrad
    from torchrec.sparse.jagged_tensor import KeyedJaggedTensor

    from two_tower_recommender_model_amd.task import TwoTower, TwoTowerTrainTask

    num_users, num_items, D, B, layers = WORKLOADS[args.workload]
    dev = torch.device("cuda", local_rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    cat_cols = ["user_id", "product_id"]
    cfgs = [EmbeddingBagConfig(name=f"t_{f}", embedding_dim=D, num_embeddings=n, feature_names=[f])
            for f, n in zip(cat_cols, (num_users, num_items))]
    ebc = EmbeddingBagCollection(tables=cfgs, device=torch.device("meta"))
    task = TwoTowerTrainTask(TwoTower(embedding_bag_collection=ebc, layer_sizes=layers, device=dev))
    _apply_optimizer_in_backward(RowWiseAdagrad, task.two_tower.ebc.parameters(), {"lr": 0.01})
    model = DistributedModelParallel(module=task, device=dev)
    optimizer = KeyedOptimizerWrapper(dict(model.named_parameters()), lambda ps: torch.optim.Adam(ps, lr=0.01))
    nb = max(2, args.batches)
    batches = []
    if args.workload in MULTIHOT:  # config 5: multi-hot bags (the KJT the reference's loader would give)
        for v, o, lab in synth_kjt_batches(num_users, num_items, B, MULTIHOT[args.workload], min(nb, 8), dev,
                                           args.ids, seed=4 * 1000 + 1 + rank):
            lengths = (o[1:] - o[:-1]).to(torch.int32)
            lpk = [int(o[B]), int(o[2 * B]) - int(o[B])]
            kjt = KeyedJaggedTensor(keys=cat_cols, values=v, lengths=lengths, offsets=o, length_per_key=lpk)
            batches.append(Batch(dense_features=torch.zeros(1, device=dev), sparse_features=kjt, labels=lab))
    else:
        for cols, lab in synth_batches(num_users, num_items, B, nb, dev, args.ids, seed=1 + 1000 * rank):
            values, lengths, offsets, lpk = ops.kjt_build_mod_dropzero(cols, [num_users, num_items])
            n = int(lpk.sum())
            kjt = KeyedJaggedTensor(keys=cat_cols, values=values[:n], lengths=lengths, offsets=offsets,
                                    length_per_key=lpk.tolist())
            batches.append(Batch(dense_features=torch.zeros(1, device=dev), sparse_features=kjt, labels=lab))
    torch.cuda.synchronize()

    def timed(pipeline, warmup, steps):
        it = itertools.cycle(batches)
        for _ in range(warmup):
            pipeline.progress(it)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            loss, _, _ = pipeline.progress(it)
        torch.cuda.synchronize()
        if world > 1:
            return end_timed_region(t0, dev)[0], float(loss)
        return time.perf_counter() - t0, float(loss)

    pipeline = TrainPipelineSparseDist(model, optimizer, dev)
    pipeline._model.train()
    dt, loss = timed(pipeline, args.warmup, args.steps)
    fd = pipeline._fused
    if world > 1 and fd:
        fd.check_errors()  # collective: a segment overflow or a multi-id bag would void the timing
    info = {"dispatch": pipeline._fused_reason, "fused_steps": fd.steps_fused if fd else 0,
            "generic_steps": fd.steps_generic if fd else args.warmup + args.steps,
            "loop": "DistributedModelParallel + TrainPipelineSparseDist.progress + KeyedOptimizerWrapper(Adam) + "
                    "RowWiseAdagrad in backward (03_model_training.py:612-625, :770-829); resident device KJTs"}
    # the same loop with the dispatch off: the generic per-op path (pooled fwd, per-layer GEMMs, dot +
    # BCE, autograd, dedup + Adagrad kernels, torch Adam) on the same storage
    os.environ["TT_DROPIN_FUSED"] = "0"
    try:
        gp = TrainPipelineSparseDist(model, optimizer, dev)
        gsteps = min(args.steps, 20)
        gdt, _ = timed(gp, 3, gsteps)
    finally:
        os.environ.pop("TT_DROPIN_FUSED", None)
    info["generic_path"] = {"ms_per_step": round(gdt / gsteps * 1e3, 4), "pairs/s": round(world * gsteps * B / gdt, 1),
                            "steps": gsteps}
    if world > 1 and fd:
        st = fd.step
        info["sharded"] = {"sharding": fd.sharding, "owners": fd.owners, "step": fd.mode,
                           "capacity": (list(st.caps_f) if fd.mode == "pipelined" else st.cap) if st is not None else None,
                           "mode": "hipgraph" if fd.graph_mode else "eager", "exchange": fd.exchange,
                           "rejected": dict(fd.rejected)}
    return world * args.steps * B / dt, dt / args.steps * 1e3, loss, args.steps, info


def run_host_fed(args):
    """The fused step fed from HOST batches (host_pipeline.HostFedPipeline): numpy columns as the
    reference's loader yields them -> pinned staging -> async H2D on a copy stream -> k-step graph
    replays; the host copies overlap the device. pairs/s over K steps (PCIe-inclusive)."""
    import itertools

    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep
    from two_tower_recommender_model_amd.host_pipeline import HostFedPipeline, synthetic_host_batches

    num_users, num_items, D, B, layers = WORKLOADS[args.workload]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    step = FusedTwoTowerStep([num_users, num_items], [D, D], [0], [1], layers, B, dev, lr_emb=0.01,
                             lr_dense=0.01, id_dtype=torch.int64, seed=0)
    host = synthetic_host_batches([num_users, num_items], B, args.batches, seed=1)
    pipe = HostFedPipeline(step, group=args.steps_per_graph or 8, depth=4, trace=True)
    src = itertools.cycle(host)
    # whole groups, and enough of them that the pipeline's fill (two groups copied before the first
    # replay) and drain do not dominate: at least 64 groups timed
    g = args.steps_per_graph or 8
    steps = max(64 * g, -(-args.steps // g) * g)
    pipe.run(src, max_steps=max(args.warmup, 4 * g))
    torch.cuda.synchronize()
    pipe.trace.clear()
    t0 = time.perf_counter()
    n = pipe.run(src, max_steps=steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    info = pipe.summary()
    info.update(graphs="production ring" if pipe.ring else "classic pool", steps_per_group=g,
                host_cpus=len(os.sched_getaffinity(0)), torch_threads=torch.get_num_threads())
    return n * B / dt, dt / n * 1e3, float(step.loss), n, info


def run_multi(args, world, rank, local_rank):
    """N >= 1 ranks, one per GPU: the pipelined sharded single-hot step (row-wise shards of both
    tables; per step one all-to-all of [gradient rows | tower gradient | next batch's ids] and one of
    the next batch's rows, over RCCL; data-parallel towers), replayed as HIP graphs with the
    collectives inside (eager launches if capture is refused). Segment capacities are sized from the
    resident batches (max over batches and ranks), so no timed step can overflow; the sticky
    overflow / bad-key flags are all-reduced and checked before and after the timed region."""
    from two_tower_recommender_model_amd.sharded import (FusedShardedTwoTowerStep, PeerComm, capture_pool_or_eager,
                                                         default_capacity, exchange_comm, segment_counts)

    N, Fq, D, B, layers, sharding, owners, ids, seed, plan = sharded_spec(args, world)
    F = len(N)
    dev = torch.device("cuda", local_rank % torch.cuda.device_count())  # (rehearsal: ranks may share one GPU)
    # the exchanges' per-destination blocks (gradient rows fp32, returned rows bf16): "auto" times
    # both exchanges on them and keeps RCCL where the device-initiated stores do not pay
    per_dest = -(-F * B // world)
    comm, xdesc = exchange_comm(args.exchange, device=dev, probe=[per_dest * D * 4, per_dest * D * 2])
    peer = isinstance(comm, PeerComm)
    k = args.steps_per_graph or 8
    nb = max(2 * k, args.batches // (2 * k) * (2 * k))  # even and a multiple of k
    batches = synth_cols(N, B, nb, dev, ids, seed=seed * 1000 + 1 + rank)
    blocks = [-(-n // world) if sh == "row_wise" else 0 for n, sh in zip(N, sharding)]
    seg_owner = [o if sh == "table_wise" else 0 for o, sh in zip(owners, sharding)]
    need = torch.zeros(1, dtype=torch.int64)
    for cols, _ in batches:
        need = torch.maximum(need, segment_counts(cols, N, blocks, seg_owner, world).max().reshape(1))
    need = need.to(dev)
    dist.all_reduce(need, op=dist.ReduceOp.MAX)
    cap = max(default_capacity(B, world), -(-int(need) // 8) * 8)
    step = FusedShardedTwoTowerStep(comm, N, D, layers, B, dev, sharding=sharding, tw_owners=owners, lr_emb=0.01,
                                    lr_dense=0.01, seed=0, capacity=cap, num_query_features=Fq,
                                    overlap=args.overlap)
    step.load_batch(*batches[0])
    step.step()  # creates the RCCL communicators before any capture
    # gloo collectives (TT_REHEARSE_GLOO, testing only) are not capturable: eager steps
    # (the device-initiated exchange is capturable whatever the backend: gloo only carries its setup)
    mode = capture_pool_or_eager(step, batches, k, allow_capture=os.environ.get("TT_REHEARSE_GLOO") != "1" or peer)

    def run(n):
        if mode == "eager":
            step.run_eager(batches, n)
        else:
            step.run(n)

    run(args.warmup)
    torch.cuda.synchronize()
    step.check()  # all ranks: a segment over capacity would invalidate the timed steps
    dist.barrier()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    dt, dt_barrier = end_timed_region(t0, dev)
    step.check()
    loss = float(step.loss)
    step.release_graphs()  # before the process group is destroyed
    r = step.rank
    if peer:
        dist.barrier()  # no rank unmaps a peer's buffer while that peer may still store into it
        comm.close()
    # SURVEY 8(d) embedding-path bytes per rank and step over the whole step's time (no per-launch
    # timing in this mode): every rank routes B x F lookups and owns ~B x F of the W x B x F lookups
    # for the update; U counted on this rank's resident batches (distinct (table, row) per batch)
    FB = F * B
    uniq = sum(int(torch.unique(torch.cat([c[f][c[f] != 0] % N[f] + (f << 40) for f in range(F)])).numel())
               for c, _ in batches) // len(batches)
    emb_bytes = FB * (16 + 4 * D) + FB * (4 + 8 * D) + uniq * (8 * D + 8)
    ach = emb_bytes / (dt / args.steps) / 1e9
    roofline = {"bound": "hbm", "kernel": "whole sharded step (per rank)", "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "alg_bytes_per_step": emb_bytes, "unique_rows": uniq,
                "timing": "SURVEY 8(d) bytes per rank over the max-over-ranks step time (collectives included)"}
    info = {"plan": plan, "features": F, "query_features": Fq, "ids": ids,
            "capacity": cap, "capacity_needed": int(need), "resident_batches": nb,
            "exchange_A_bytes_sent": 4 * step.A_total,
            "exchange_B_bytes_sent": 2 * D * world * step.S[r],
            "collectives_per_step": 2, "mode": mode,
            "ms_per_step_with_closing_barrier": round(dt_barrier / args.steps * 1e3, 5),
            "exchange": xdesc + ("; producers store at the destinations" if getattr(step, "direct", False) else "")
                        + ("; launch U / Adam signal and wait in-launch" if getattr(step, "merged", False) else ""),
            "overlap": "T2 (tower weight gradients) on a parallel graph branch beside exchange A + the owner's "
                       "update" if step.overlap else "none (one stream)"}
    return world * args.steps * B / dt, dt / args.steps * 1e3, loss, info, roofline


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` started without a launcher: run the same command line as N ranks under
    `torch.distributed.run` (one process per GPU, the reference's TorchDistributor(num_processes=N)
    at 03_model_training.py:918) in a CHILD process, stdout / stderr inherited (rank 0's JSON line
    passes straight through), and return its exit status. This process never touches the GPU:
    torch.cuda.device_count() does not initialise HIP on this stack, and nothing else here does."""
    import subprocess

    rehearse = os.environ.get("TT_REHEARSE_GLOO") == "1"  # testing only: ranks share the visible GPUs
    have = torch.cuda.device_count()
    if not rehearse and have < n:
        print(f"bench.py --gpus {n}: only {have} GPU(s) visible (one process per GPU)", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" in os.environ and world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} under a launcher of world size {world}: they must agree")
    if args.ids is None:
        args.ids = SHARDED[args.workload]["ids"] if args.workload in SHARDED else "uniform"
    if args.workload in SHARDED:
        sp = SHARDED[args.workload]
        D, B, layers = sp["D"], sp["B"], sp["layers"]
        desc = {"config3": "16 single-hot tables, 8 features per tower (user_id 50M, product_id 100M, 14 x 1M)",
                "config4": "1B-row product_id table (row-wise) x 50M-row user_id table (table-wise)"}[args.workload]
        config = {"workload": f"{args.workload}: {desc}, emb_dim {D}, towers {layers}, {args.ids} ids",
                  "global_batch": B * world, "per_gpu_batch": B, "emb_dim": D,
                  "tower_dtype": "bf16 (MFMA, fp32 acc)"}
    else:
        num_users, num_items, D, B, layers = WORKLOADS[args.workload]
        hot = f"multi-hot (bags of 1..{MULTIHOT[args.workload]})" if args.workload in MULTIHOT else "single-hot"
        config = {"workload": f"{args.workload}: {num_items // 1_000_000}M items x {num_users // 1_000_000}M users, "
                              f"emb_dim {D}, towers {layers}, {hot} {args.ids} ids",
                  "global_batch": B * world, "per_gpu_batch": B, "emb_dim": D, "tower_dtype": "bf16 (MFMA, fp32 acc)",
                  "parallelism": "single-gpu hipgraph"}
    sharded_info = None
    if args.workload in MULTIHOT and world == 1 and not args.sharded:
        value, ms, loss, roofline, cpu, steps_run = run_multihot(args)
        config["parallelism"] = "single-gpu hipgraph, KJT input"
    elif world == 1 and args.path == "dropin":
        value, ms, loss, steps_run, di = run_dropin(args)
        roofline, cpu = None, None
        config["dropin"] = di
        config["parallelism"] = "single-gpu: the reference's DMP + TrainPipelineSparseDist loop, dispatched to the fused ring"
    elif world == 1 and args.host_fed:
        value, ms, loss, steps_run, hf = run_host_fed(args)
        roofline, cpu = None, None
        config["host_fed"] = hf
        config["parallelism"] = "single-gpu, host-fed: pinned staging + async H2D (copy stream) + hipgraph replay"
        config["note"] = "PCIe-inclusive rate (inputs handed over in host memory); the resident-input line is the metric"
    elif world == 1 and not args.sharded and args.workload not in SHARDED:
        value, ms, loss, roofline, cpu, steps_run = run_single(args)
    else:
        # TT_REHEARSE_GLOO=1 (testing only, never a bench line): gloo collectives and ranks sharing the
        # visible GPUs, to run the N > 1 code path (routes, capacities, flags, eager collectives) on a
        # one-GPU box; the production path is RCCL, one GPU per rank
        rehearse = os.environ.get("TT_REHEARSE_GLOO") == "1"
        if rehearse:
            local_rank = local_rank % torch.cuda.device_count()
        torch.cuda.set_device(local_rank)
        from two_tower_recommender_model_amd.sharded import graph_safe_nccl_env

        graph_safe_nccl_env()  # RCCL collectives inside HIP graphs (before the process group exists)
        if rehearse:
            dist.init_process_group("gloo")
        elif "RANK" in os.environ:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:  # --sharded without a launcher (e.g. under rocprofv3): a one-rank group
            dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(),
                                    device_id=torch.device("cuda", local_rank))
        if args.path == "dropin":
            value, ms, loss, steps_run, di = run_dropin(args, world, rank, local_rank)
            config["dropin"] = di
            config["parallelism"] = (f"the reference's DMP + TrainPipelineSparseDist loop x{world}, dispatched to the "
                                     f"fused sharded step")
            roofline, sharded_info = None, di.get("sharded")
        elif args.workload in MULTIHOT:
            value, ms, loss, sharded_info, roofline = run_multi_kjt(args, world, rank, local_rank)
            xk = "RCCL" if sharded_info["exchange"].startswith("RCCL") else "device-initiated"
            config["parallelism"] = (f"{sharded_info['plan']} + data-parallel towers x{world}: 3 fixed-size {xk} "
                                     f"all-to-alls per step (ids, pooled rows, bag gradients), {sharded_info['mode']}")
        else:
            value, ms, loss, sharded_info, roofline = run_multi(args, world, rank, local_rank)
            xk = "RCCL" if sharded_info["exchange"].startswith("RCCL") else "device-initiated"
            config["parallelism"] = (f"{sharded_info['plan']} sharded tables + data-parallel towers x{world}: pipelined, "
                                     f"2 {xk} all-to-alls per "
                                     f"step ([grad rows | tower grad | next ids], next rows), "
                                     f"{sharded_info['mode']}")
        cpu, steps_run = None, args.steps
        config["sharded"] = sharded_info
    if rank == 0:
        out = {"metric": f"training pairs/sec at batch {B} (per GPU)", "value": round(value, 1), "unit": "pairs/s",
               "n_gpus": world, "steps": steps_run, "warmup": args.warmup, "ms_per_step": round(ms, 5),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
               "data": f"synthetic ({args.ids} ids, Bernoulli labels), random-init weights", "config": config,
               "loss": loss, "roofline": roofline, "cpu_baseline": cpu}
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
