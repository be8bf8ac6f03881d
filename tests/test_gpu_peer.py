"""The device-initiated exchange (sharded.PeerComm, csrc/peer.hip) against torch.distributed on the
sharded step, bit for bit (tests/peer_xchg_check.py): at world 1 in one process, and at world 2 as two
processes sharing the test box's GPU, each rank's puts landing in the other process's receive buffers
through hipIpcOpenMemHandle. The cross-device (xGMI) form is the driver's multi-GPU node's."""
import os

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_peer_exchange_world1_graph_equals_sync_steps():
    from child_util import run_child

    run_child(["tests/peer_xchg_check.py"], "PEER-XCHG-OK world 1", timeout=150)


def test_peer_exchange_two_processes_equal_gloo():
    from child_util import run_child

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    run_child(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
               "--master-port", "29571", "tests/peer_xchg_check.py"], "PEER-XCHG-OK world 2", timeout=170, env=env)
