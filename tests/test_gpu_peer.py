"""The device-initiated exchange (sharded.PeerComm, csrc/peer.hip) against torch.distributed on the
sharded step, bit for bit (tests/peer_xchg_check.py): at world 1 in one process, and at world 2 as two
processes sharing the test box's GPU, each rank's puts landing in the other process's receive buffers
through hipIpcOpenMemHandle. The cross-device (xGMI) form is the driver's multi-GPU node's."""
import os

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# "system": TT_PEER_SYSTEM_SCOPE=1 forces the signalling ranks on different GPUs use (system-scope
# release / acquire, fine-grained memory required) onto these same-GPU ranks
SCOPES = {"agent": {}, "system": {"TT_PEER_SYSTEM_SCOPE": "1"}}


@pytest.mark.parametrize("scope", sorted(SCOPES))
def test_peer_exchange_world1_graph_equals_sync_steps(scope):
    from child_util import run_child

    run_child(["tests/peer_xchg_check.py"], "PEER-XCHG-OK world 1", timeout=150,
              env=dict(os.environ, **SCOPES[scope]))


@pytest.mark.parametrize("scope", sorted(SCOPES))
def test_peer_exchange_two_processes_equal_gloo(scope):
    from child_util import run_child

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(SCOPES[scope])
    run_child(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
               "--master-port", "29571", "tests/peer_xchg_check.py"], "PEER-XCHG-OK world 2", timeout=170, env=env)
