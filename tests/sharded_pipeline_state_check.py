"""Child process of tests/test_gpu_sharded.py::test_sharded_pipeline_state_resets (one-rank RCCL group).

(1) A pool capture refused after its first captured step (the production fallback,
    ``capture_pool_or_eager``): the eager steps that follow must equal a run that never tried to
    capture, bit for bit (the refused capture primed batch 0 into a dedup table; priming it again
    without a reset would file the same keys twice and those rows would never be updated).
(2) ``load_state_dict`` in the middle of a graphed run: the next ``run`` re-primes from the loaded
    weights and equals an eager run from the same state, bit for bit.
The failure is injected by replacing the step's ``step_pipelined`` on the instance (test only)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from two_tower_recommender_model_amd import _lib  # noqa: E402
from two_tower_recommender_model_amd.sharded import (FusedShardedTwoTowerStep, ThreadComm, TorchComm,  # noqa: E402
                                                     capture_pool_or_eager, graph_safe_nccl_env)


def same(a, b):
    return (torch.equal(a.tables.weights, b.tables.weights) and torch.equal(a.tables.state, b.tables.state)
            and torch.equal(a.params, b.params) and torch.equal(a.exp_avg_sq, b.exp_avg_sq)
            and float(a.loss) == float(b.loss))


def main():
    device = torch.device("cuda:0")
    torch.cuda.set_device(device)
    from child_util import seed_all

    seed_all(0)
    graph_safe_nccl_env()
    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(), device_id=device)
    B, D, N = 1024, 128, [20_000, 30_000]
    g = torch.Generator().manual_seed(7)
    batches = []
    for _ in range(4):
        cols = [torch.randint(0, n, (B,), generator=g).to(device) for n in N]
        cols[1][:24] = 555  # a row looked up many times
        batches.append((cols, torch.randint(0, 2, (B,), generator=g).to(torch.int32).to(device)))
    full = [torch.empty(n, D).uniform_(-0.01, 0.01, generator=g) for n in N]

    def make(comm):
        st = FusedShardedTwoTowerStep(comm, N, D, [128, 64], B, device, full_tables=full, seed=4)
        st.load_batch(*batches[0])
        st.step()  # (RCCL: communicator init before any capture)
        return st

    ok = True
    # ---- (1) refused capture -> eager fallback
    a = make(TorchComm(always_collective=True))
    real = a.step_pipelined
    calls = [0]

    def failing(*args, **kw):
        real(*args, **kw)
        calls[0] += 1
        if torch.cuda.is_current_stream_capturing() and calls[0] >= 1:
            raise _lib.TTError("capture refused (test injection)")

    a.step_pipelined = failing
    mode = capture_pool_or_eager(a, batches, 2)
    a.step_pipelined = real
    a.run_eager(batches, 6)
    b = make(ThreadComm.group(1)[0])
    b.run_eager(batches, 6)
    torch.cuda.synchronize()
    a.check()
    r1 = mode == "eager" and same(a, b)
    print(f"fallback mode={mode} equal={r1}", flush=True)
    ok &= r1
    a.release_graphs()
    # ---- (2) load_state_dict in the middle of a graphed run
    c = make(TorchComm(always_collective=True))
    c.capture_pool(batches, steps_per_graph=2)
    c.run(3)
    sd = c.gathered_state_dict(optimizer=True)
    sd = {k: v.clone() for k, v in sd.items()}
    c.run(2)  # progress past the checkpoint: staged rows and dedup tables now belong to other batches
    c.load_state_dict(sd)
    c.run(3)  # re-primes at the pool's batch 0
    d = make(ThreadComm.group(1)[0])
    d.run_eager(batches, 3)
    d.reset_pipeline()
    d.run_eager(batches, 3)
    torch.cuda.synchronize()
    c.check()
    r2 = same(c, d)
    print(f"resume equal={r2}", flush=True)
    ok &= r2
    c.release_graphs()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("PIPELINE-STATE-OK" if ok else "PIPELINE-STATE-MISMATCH", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    from child_util import child_main

    child_main(main)
