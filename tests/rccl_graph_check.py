"""Child process of tests/test_gpu_sharded.py::test_sharded_rccl_world1_graph_equals_eager."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from two_tower_recommender_model_amd.sharded import (FusedShardedTwoTowerStep, ThreadComm, TorchComm,  # noqa: E402
                                                     graph_safe_nccl_env)


def main():
    device = torch.device("cuda:0")
    torch.cuda.set_device(device)
    from child_util import seed_all

    seed_all(0)
    graph_safe_nccl_env()
    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(), device_id=device)
    B, D, N = 1024, 128, [30_000, 50_000]
    g = torch.Generator().manual_seed(5)
    batches = []
    for _ in range(4):
        cols = [torch.randint(0, n, (B,), generator=g).to(device) for n in N]
        batches.append((cols, torch.randint(0, 2, (B,), generator=g).to(torch.int32).to(device)))
    full = [torch.empty(n, D).uniform_(-0.01, 0.01, generator=g) for n in N]
    a = FusedShardedTwoTowerStep(TorchComm(always_collective=True), N, D, [128, 64], B, device, full_tables=full)
    b = FusedShardedTwoTowerStep(ThreadComm.group(1)[0], N, D, [128, 64], B, device, full_tables=full)
    a.load_batch(*batches[0])
    a.step()  # communicator init (eager collectives, retired by capture_pool); the same on b
    b.load_batch(*batches[0])
    b.step()
    a.capture_pool(batches, steps_per_graph=2)
    a.run(4)
    for cols, lab in batches:
        b.load_batch(cols, lab)
        b.step()
    torch.cuda.synchronize()
    a.check()
    ok = torch.equal(a.tables.weights, b.tables.weights) and torch.equal(a.params, b.params) and \
        float(a.loss) == float(b.loss)
    # teardown in order: graphs (they reference the communicator's work), then the process group
    a.release_graphs()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("RCCL-GRAPH-OK" if ok else "RCCL-GRAPH-MISMATCH", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    from child_util import child_main

    child_main(main)
