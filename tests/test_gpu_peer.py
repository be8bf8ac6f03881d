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
# world 1: "in-launch" has launch U and Adam signal / wait themselves (tt_peer_wait_t, opt-in
# TT_PEER_MERGED=1); "kernels" the separate signal / wait kernels (the default)
WAITS = {"in-launch": {"TT_PEER_MERGED": "1", "TT_PEER_EXPECT_MERGED": "1"},
         "kernels": {"TT_PEER_MERGED": "0", "TT_PEER_EXPECT_MERGED": "0"}}


@pytest.mark.parametrize("waits", sorted(WAITS))
@pytest.mark.parametrize("scope", sorted(SCOPES))
def test_peer_exchange_world1_graph_equals_sync_steps(scope, waits):
    from child_util import run_child

    run_child(["tests/peer_xchg_check.py"], "PEER-XCHG-OK world 1", timeout=150,
              env=dict(os.environ, **SCOPES[scope], **WAITS[waits]))


@pytest.mark.parametrize("scope", sorted(SCOPES))
def test_peer_exchange_two_processes_equal_gloo(scope):
    from child_util import run_child

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(SCOPES[scope])
    env.update(TT_PEER_MERGED="1", TT_PEER_EXPECT_MERGED="0")  # ranks sharing the GPU: never in-launch waits
    run_child(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
               "--master-port", "29571", "tests/peer_xchg_check.py"], "PEER-XCHG-OK world 2", timeout=170, env=env)
