"""Child process of tests/test_gpu_peer.py: the sharded step with PeerComm (device-initiated exchange
into IPC-mapped peer buffers, csrc/peer.hip) against the same step over torch.distributed.

World 1 (no launcher): a one-rank gloo group; the PeerComm step runs its pipelined pool as HIP graphs,
the reference step is ThreadComm's synchronous step() over the same batches. World W (under
torch.distributed.run, gloo, ranks sharing the GPU): every rank runs the PeerComm step as graphs and
a TorchComm (gloo, eager) step with run_eager over the same batches. Bit for bit on every rank: the
rank's table shards, tower parameters, loss; and no wait timed out (check())."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from child_util import stage  # noqa: E402
from two_tower_recommender_model_amd.sharded import (FusedShardedTwoTowerStep, PeerComm, ThreadComm,  # noqa: E402
                                                     TorchComm)


def main():
    device = torch.device("cuda:0")
    torch.cuda.set_device(device)
    launched = "WORLD_SIZE" in os.environ
    if launched:
        dist.init_process_group("gloo")
    else:
        dist.init_process_group("gloo", rank=0, world_size=1, store=dist.HashStore())
    W, r = dist.get_world_size(), dist.get_rank()
    B, D, N = 1024, 128, [30_000, 50_000]
    steps = int(os.environ.get("TT_PEER_STEPS", "8"))
    g = torch.Generator().manual_seed(5)
    full = [torch.empty(n, D).uniform_(-0.01, 0.01, generator=g) for n in N]
    g = torch.Generator().manual_seed(100 + r)
    batches = []
    for _ in range(4):
        cols = [torch.randint(0, n, (B,), generator=g).to(device) for n in N]
        batches.append((cols, torch.randint(0, 2, (B,), generator=g).to(torch.int32).to(device)))
    cap = 2048  # per (owner, feature) segment: >= the ~B / W + noise any batch sends one owner
    stage("peer comm")
    pc = PeerComm(timeout_s=5.0, device=device)
    ok, why = pc.self_test()  # the startup check exchange_comm runs before trusting the protocol
    print(f"rank {r}: self-test ok {ok} ({why}), same_device {pc.same_device}", flush=True)
    assert ok, why
    a = FusedShardedTwoTowerStep(pc, N, D, [128, 64], B, device, full_tables=full, capacity=cap)
    ref_comm = TorchComm() if launched else ThreadComm.group(1)[0]
    b = FusedShardedTwoTowerStep(ref_comm, N, D, [128, 64], B, device, full_tables=full, capacity=cap)
    print(f"rank {r}: PeerComm memory {pc.memory}, direct {a.direct}, in-launch waits {a.merged}", flush=True)
    if os.environ.get("TT_PEER_EXPECT_MERGED"):
        assert a.merged == (os.environ["TT_PEER_EXPECT_MERGED"] == "1"), "in-launch waits not as expected"
    stage("synchronous step")
    a.load_batch(*batches[0])
    a.step()
    b.load_batch(*batches[0])
    b.step()
    torch.cuda.synchronize()
    ok = torch.equal(a.tables.weights, b.tables.weights) and torch.equal(a.params, b.params)
    stage("graphs")
    a.capture_pool(batches, steps_per_graph=2)
    dist.barrier()
    a.run(steps)
    torch.cuda.synchronize()
    stage("reference")
    if launched:
        b.run_eager(batches, steps)
    else:
        for i in range(steps):
            b.load_batch(*batches[i % len(batches)])
            b.step()
    torch.cuda.synchronize()
    a.check()
    ok = ok and torch.equal(a.tables.weights, b.tables.weights) and torch.equal(a.params, b.params) and \
        float(a.loss) == float(b.loss)
    print(f"rank {r}: loss {float(a.loss):.6f} vs {float(b.loss):.6f}, equal {ok}", flush=True)
    okt = torch.tensor([1 if ok else 0])
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    a.release_graphs()
    torch.cuda.synchronize()
    dist.barrier()
    pc.close()
    dist.destroy_process_group()
    if r == 0:
        print(f"PEER-XCHG-OK world {W}" if int(okt) else "PEER-XCHG-MISMATCH", flush=True)
    return 0 if int(okt) else 1


if __name__ == "__main__":
    from child_util import child_main

    child_main(main)
