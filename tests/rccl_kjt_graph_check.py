"""Child of tests/test_gpu_sharded_kjt.py::test_sharded_kjt_rccl_world1_graph_equals_eager: the multi-hot
sharded step with its three all-to-alls on RCCL (a one-rank "nccl" group, collectives forced on),
captured into HIP graphs over resident batches, equals the same steps run eagerly, bit for bit.
With TT_KJT_COMM=peer the graphs run on sharded.PeerComm (device-initiated puts) against the eager
RCCL steps. Prints RCCL-KJT-GRAPH-OK."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from child_util import seed_all, stage  # noqa: E402


def main():
    device = torch.device("cuda:0")
    torch.cuda.set_device(device)
    seed_all(0)
    from two_tower_recommender_model_amd.sharded import TorchComm, graph_safe_nccl_env

    graph_safe_nccl_env()
    stage("init_process_group")
    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(), device_id=device)
    from two_tower_recommender_model_amd.sharded_kjt import FusedShardedKJTStep

    N, B, D = [3000, 5000], 512, 128
    g = torch.Generator().manual_seed(9)
    full = [torch.empty(n, D).uniform_(-0.05, 0.05, generator=g) for n in N]
    batches = []
    for _ in range(4):
        lengths = torch.randint(0, 12, (2 * B,), generator=g).to(torch.int32)
        vals = torch.cat([torch.randint(0, N[i // B], (int(lengths[i]),), generator=g) for i in range(2 * B)])
        offs = torch.zeros(2 * B + 1, dtype=torch.int32)
        offs[1:] = torch.cumsum(lengths, 0)
        batches.append((vals.to(torch.int32).to(device), offs.to(device),
                        torch.randint(0, 2, (B,), generator=g).to(torch.int32).to(device)))
    cap = max(int(v.numel()) for v, _, _ in batches)
    mk = lambda comm: FusedShardedKJTStep(comm, N, D, [128, 64], B, device, cap=cap,  # noqa: E731
                                          sharding=("table_wise", "row_wise"), tw_owners=(0, 0), full_tables=full)
    stage("eager")
    a = mk(TorchComm(always_collective=True))
    for v, o, l in batches + batches[:2]:
        a.step(v, o, l)
    torch.cuda.synchronize()
    stage("graphs")
    peer = os.environ.get("TT_KJT_COMM") == "peer"  # the graphs over the device-initiated exchange
    if peer:
        from two_tower_recommender_model_amd.sharded import PeerComm

        pc = PeerComm(device=device)
    b = mk(pc if peer else TorchComm(always_collective=True))
    b.capture_pool(batches)
    b.run(6)
    torch.cuda.synchronize()
    a.check()
    b.check()
    for f in range(2):
        assert torch.equal(a.tables.table_view(f), b.tables.table_view(f)), f
        assert torch.equal(a.tables.state_view(f), b.tables.state_view(f)), f
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.logits, b.logits)
    b.release_graphs()
    del a, b
    torch.cuda.synchronize()
    if peer:
        pc.close()
    dist.destroy_process_group()
    print("RCCL-KJT-GRAPH-OK", flush=True)
    return 0


if __name__ == "__main__":
    from child_util import child_main

    child_main(main)
