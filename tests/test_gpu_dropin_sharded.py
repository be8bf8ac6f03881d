"""The reference's loop at world size W > 1 dispatched to the fused sharded step
(two_tower_recommender_model_amd/dropin.py FusedShardedDropin; 03_model_training.py:812-815, :648):
W processes under torch.distributed.run share the test box's one MI355X over gloo
(tests/dropin_sharded_check.py). The production run is RCCL with one GPU per rank, where the step's
all-to-alls are captured into the slot graphs.

* bitwise: the drop-in equals FusedShardedTwoTowerStep run directly on the same initial shards,
  towers and capacity, bit for bit (per-step logits / loss; every rank's shards, row-wise Adagrad
  state, tower parameters and Adam moments), for the default plan (both tables row-wise), both
  tables table-wise and the mixed plan;
* mixed: a smaller batch in the middle runs the generic DMP path on every rank and the fused
  steps re-prime after it; eval runs forward-only."""
import os
import socket
import sys

import pytest

from child_util import run_child

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, *args):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    argv = ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world), "--master-addr",
            "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tests", "dropin_sharded_check.py"),
            *args]
    run_child(argv, "DROPIN-SHARDED-OK", timeout=150, env=env)


@pytest.mark.parametrize("world,plan", [(2, "default"), (2, "tw"), (3, "mixed")])
def test_dropin_sharded_bitwise_equals_direct_step(world, plan):
    _run(world, "--mode", "bitwise", "--plan", plan)


def test_dropin_sharded_generic_batch_and_eval():
    _run(2, "--mode", "mixed", "--plan", "mixed", "--dim", "64")
