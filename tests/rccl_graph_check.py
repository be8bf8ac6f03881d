"""Child process of tests/test_gpu_sharded.py::test_sharded_rccl_world1_graph_equals_eager."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from two_tower_recommender_model_amd.sharded import (FusedShardedTwoTowerStep, ThreadComm, TorchComm,  # noqa: E402
                                                     graph_safe_nccl_env)


def main():
    device = torch.device("cuda:0")
    torch.cuda.set_device(device)
    graph_safe_nccl_env()
    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(), device_id=device)
    B, D, N = 1024, 128, [30_000, 50_000]
    g = torch.Generator().manual_seed(5)
    batches = []
    for _ in range(4):
        cols = [torch.randint(0, n, (B,), generator=g).to(device) for n in N]
        batches.append((cols, torch.randint(0, 2, (B,), generator=g).to(torch.int32).to(device)))
    full = [torch.empty(n, D).uniform_(-0.01, 0.01, generator=g) for n in N]
    a = FusedShardedTwoTowerStep(TorchComm(always_collective=True), N, D, [128, 64], B, device, full_tables=full,
                                 overlap_comm="--overlap" in sys.argv)
    b = FusedShardedTwoTowerStep(ThreadComm.group(1)[0], N, D, [128, 64], B, device, full_tables=full)
    a.load_batch(*batches[0])
    a.step()  # communicator init; the same first step on b
    b.load_batch(*batches[0])
    b.step()
    torch.cuda.synchronize()
    time.sleep(0.5)  # the watchdog retires the eager collectives before the capture
    a.capture_pool(batches, steps_per_graph=2)
    for j in range(2):
        a.pool_graphs[j].replay()
    for cols, lab in batches:
        b.load_batch(cols, lab)
        b.step()
    torch.cuda.synchronize()
    a.check()
    ok = torch.equal(a.tables.weights, b.tables.weights) and torch.equal(a.params, b.params) and \
        float(a.loss) == float(b.loss)
    a.release_graphs()
    torch.cuda.synchronize()
    print("RCCL-GRAPH-OK" if ok else "RCCL-GRAPH-MISMATCH", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    rc = main()
    sys.stdout.flush()
    sys.stderr.flush()
    # the verdict is printed; leave without the communicator / HIP-graph teardown at interpreter
    # exit (one run of this child aborted there, after the comparison, with SIGABRT)
    os._exit(rc)
