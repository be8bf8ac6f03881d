"""The N > 1 bench path (bench.py run_multi: one process per rank, row-wise shards, routes,
capacities sized from the resident batches and all-reduced, sticky flags checked on every rank, the
sharded roofline line) as two real processes under torch.distributed.run on the one GPU of the test
box: TT_REHEARSE_GLOO=1 swaps RCCL for gloo (eager collectives, ranks share the GPU). The production
run is RCCL with one GPU per rank (the driver's 8-GPU node); this guards everything around it."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [2, 4])
def test_bench_multiprocess_gloo_rehearsal(world):
    env = dict(os.environ, TT_REHEARSE_GLOO="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(29517 + world), "bench.py", "--gpus", str(world),
           "--workload", "config2", "--steps", "4", "--warmup", "2", "--batches", "8", "--no-cpu-baseline",
           "--exchange", "rccl"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == world and d["steps"] == 4 and d["value"] > 0
    sh = d["config"]["sharded"]
    assert sh["mode"] == "eager" and sh["capacity"] >= sh["capacity_needed"]
    assert d["roofline"]["alg_bytes_per_step"] > 0 and d["loss"] == d["loss"]  # finite



def test_bench_gpus2_self_launch_as_driver_runs_it():
    """`python bench.py --gpus 2` with no launcher (the driver's form for the N-GPU line): the parent
    starts torch.distributed.run with 2 ranks as a child, the ranks form a world of 2 (asserted in
    bench.py against --gpus), rank 0's JSON line reaches the parent's stdout and the rc is 0."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TT_REHEARSE_GLOO="1")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "4", "--warmup", "2", "--batches", "8",
           "--workload", "config2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["value"] > 0
    assert d["config"]["global_batch"] == 2 * d["config"]["per_gpu_batch"]
    assert d["config"]["sharded"]["plan"].startswith("table-wise")
    # the default exchange: the device-initiated one after its self-test, captured into graphs
    assert d["config"]["sharded"]["exchange"].startswith("device-initiated"), d["config"]["sharded"]
    assert d["config"]["sharded"]["mode"] == "hipgraph"


def test_bench_gpus2_northstar_table_wise_as_driver_runs_it():
    """The driver's N = 2 line on the north star itself (`bench.py --gpus 2`, defaults: 100M x 50M
    tables, D 128, B 8192 per rank): table-wise plan (users on rank 0, items on rank 1, 76.8 GB on the
    shared GPU), the default exchange (device-initiated after its self-test), HIP graphs, flags
    checked on both ranks, one JSON line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TT_REHEARSE_GLOO="1")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "16", "--warmup", "4", "--batches", "16",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    print(lines[0][:600], flush=True)
    sh = d["config"]["sharded"]
    assert d["n_gpus"] == 2 and d["config"]["per_gpu_batch"] == 8192 and d["config"]["emb_dim"] == 128
    assert d["config"]["workload"].startswith("northstar")
    assert sh["plan"].startswith("table-wise") and sh["mode"] == "hipgraph", sh
    assert sh["exchange"].startswith("device-initiated"), sh
    assert d["value"] > 0 and d["loss"] == d["loss"]


def test_bench_gpus4_northstar_row_wise_peer_rehearsal():
    """The driver's N = 4 line on the north star (`bench.py --gpus 4`): the row-wise plan (both
    tables split in 4 blocks, 19.2 GB per rank on the shared GPU), four processes storing straight
    into each other's IPC-mapped exchange buffers (the default exchange after its self-test), HIP
    graphs, flags checked on every rank, one JSON line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TT_REHEARSE_GLOO="1")
    cmd = [sys.executable, "bench.py", "--gpus", "4", "--steps", "16", "--warmup", "4", "--batches", "16",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=250)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    print(lines[0][:600], flush=True)
    sh = d["config"]["sharded"]
    assert d["n_gpus"] == 4 and d["config"]["per_gpu_batch"] == 8192
    assert sh["plan"].startswith("row-wise") and sh["mode"] == "hipgraph", sh
    assert sh["exchange"].startswith("device-initiated") and "producers store" in sh["exchange"], sh
    assert d["value"] > 0 and d["loss"] == d["loss"]


def test_bench_dropin_n2_rehearsal():
    """`bench.py --gpus 2 --path dropin`: the reference's DMP + TrainPipelineSparseDist loop in two
    processes (gloo, sharing the GPU) dispatched to the fused sharded step on every rank."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TT_REHEARSE_GLOO="1")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--path", "dropin", "--workload", "config2", "--steps", "6",
           "--warmup", "2", "--batches", "8", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["loss"] == d["loss"]
    di = d["config"]["dropin"]
    assert di["dispatch"] == "fused sharded" and di["fused_steps"] == 8 and di["generic_steps"] == 0, di


def test_bench_dropin_config5_n2_dispatches_kjt_step():
    """`bench.py --gpus 2 --path dropin --workload config5`: the reference's loop on multi-hot bags
    (BASELINE config 5: B = 16,384, bags of 1..39 ids, 100M x 50M tables) in two processes sharing
    the GPU, dispatched to the fused sharded KJT step on every rank: no generic step, no rejection."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TT_REHEARSE_GLOO="1")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--path", "dropin", "--workload", "config5", "--steps", "6",
           "--warmup", "2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=230)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    print(line[:1500], flush=True)
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["loss"] == d["loss"]
    di = d["config"]["dropin"]
    assert di["dispatch"] == "fused sharded" and di["fused_steps"] == 8 and di["generic_steps"] == 0, di
    assert di["sharded"]["step"] == "kjt" and not di["sharded"]["rejected"], di


@pytest.mark.parametrize("world", [2])
def test_bench_config5_sharded_multiprocess_gloo_rehearsal(world):
    """bench.py's config-5 N > 1 path (the capturable multi-hot sharded step: users table-wise on the
    last rank, items row-wise, BASELINE table sizes and B = 16,384) as real processes over gloo
    (eager collectives, ranks sharing the one GPU): capacities all-reduced, flags checked, the line."""
    env = dict(os.environ, TT_REHEARSE_GLOO="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(29537 + world), "bench.py", "--gpus", str(world),
           "--workload", "config5", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--exchange", "rccl"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert d["n_gpus"] == world and d["steps"] == 2 and d["value"] > 0 and d["loss"] == d["loss"]
    sh = d["config"]["sharded"]
    assert sh["mode"] == "eager" and sh["collectives_per_step"] == 3


def test_bench_gpus2_peer_exchange_rehearsal():
    """`bench.py --gpus 2 --exchange peer` (the driver's form, gloo rehearsal: ranks sharing the GPU):
    the sharded step's two exchanges as device-initiated puts into the other process's IPC-mapped
    buffers, captured into HIP graphs (gloo only carries the setup), flags checked on every rank."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TT_REHEARSE_GLOO="1")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--exchange", "peer", "--steps", "8", "--warmup", "2",
           "--batches", "8", "--steps-per-graph", "2", "--workload", "config2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    sh = d["config"]["sharded"]
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["loss"] == d["loss"]
    assert sh["mode"] == "hipgraph" and sh["exchange"].startswith("device-initiated"), sh


def test_bench_config5_peer_exchange_rehearsal():
    """`bench.py --gpus 2 --workload config5 --exchange peer` (gloo rehearsal, ranks sharing the GPU): the
    multi-hot sharded step's three exchanges as device-initiated puts, captured into HIP graphs."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TT_REHEARSE_GLOO="1")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--workload", "config5", "--exchange", "peer", "--steps", "4",
           "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    sh = d["config"]["sharded"]
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["loss"] == d["loss"]
    assert sh["mode"] == "hipgraph" and sh["exchange"].startswith("device-initiated"), sh


def test_bench_sharded_world1_probes_the_exchange():
    """`bench.py --sharded` at world 1 (backend "nccl"): exchange_comm("auto") runs the PeerComm
    self-test, then times both exchanges on the step's block sizes and keeps the faster; the line
    names the choice and both probe times, and the step runs as HIP graphs."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT",
                                                              "TT_REHEARSE_GLOO")}
    cmd = [sys.executable, "bench.py", "--sharded", "--steps", "8", "--warmup", "2", "--batches", "8",
           "--steps-per-graph", "2", "--workload", "config2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    sh = d["config"]["sharded"]
    assert d["n_gpus"] == 1 and d["value"] > 0 and sh["mode"] == "hipgraph", sh
    assert "probe" in sh["exchange"] and "against RCCL" in sh["exchange"], sh["exchange"]
