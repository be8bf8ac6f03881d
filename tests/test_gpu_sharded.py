"""The sharded single-hot step (two_tower_recommender_model_amd/sharded.py, csrc/shard.hip) on one
GPU: the route kernel against the oracle restatement (bit-exact), the whole step at W = 1 against
the single-GPU fused step (bit-exact), and W = 2 / 3 ranks run as threads of this process over an
in-process all-to-all (ThreadComm) against the oracle: the rows each rank's towers read equal the
oracle tables bit for bit, every shard after each step equals the oracle's row-wise Adagrad over
the union of the gradient rows the ranks produced (ascending (rank, bag) order), and the
data-parallel towers stay identical on every rank."""
import threading

import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,mode", [(1, "rw"), (2, "rw"), (3, "mix"), (8, "rw"), (5, "tw")])
@pytest.mark.parametrize("dtype", [torch.int64, torch.int32])
def test_route_kernel_vs_oracle(device, W, mode, dtype):
    import ctypes as C

    from two_tower_recommender_model_amd import _lib
    from two_tower_recommender_model_amd._lib import id_dtype_code, ptr, ptr_array, stream_handle

    g = torch.Generator().manual_seed(W)
    B, N = 9000, [50_000, 7_777]  # a ragged last workgroup of the route kernels
    cols = [torch.randint(-2 * n, 3 * n, (B,), generator=g) for n in N]
    for c in cols:
        c[torch.rand(B, generator=g) < 0.05] = 0
    bs = [-(-n // W) for n in N] if mode == "rw" else ([-(-N[0] // W), 0] if mode == "mix" else [0, 0])
    ow = [0, W - 1] if mode != "rw" else [0, 0]
    C_ = B if W == 1 else int(1.25 * B / W) + 64
    send = torch.zeros(W, 2 + 2 * C_, dtype=torch.int64, device=device)
    pos = torch.zeros(2 * B, dtype=torch.int32, device=device)
    flags = torch.zeros(2, dtype=torch.int32, device=device)
    dcols = [c.to(dtype).to(device) for c in cols]
    lib = _lib.load()
    ws = torch.empty(lib.tt_shard_route_workspace_bytes(2, B), dtype=torch.uint8, device=device)
    _lib.check(lib.tt_shard_route_cols(2, B, ptr_array(dcols), id_dtype_code(dtype), (C.c_int64 * 2)(*N),
                                       (C.c_int64 * 2)(*bs), (C.c_int32 * 2)(*ow), W, C_, ptr(send), ptr(pos),
                                       ptr(flags), ptr(ws), ws.numel(), stream_handle(device)))
    torch.cuda.synchronize()
    want_send, want_pos, ovf = ref.shard_route([c.numpy() for c in cols], N, bs, ow, W, C_)
    assert bool(flags[0]) == ovf
    np.testing.assert_array_equal(pos.cpu().numpy(), want_pos)
    s = send.cpu().numpy()
    for d in range(W):
        for f in range(2):
            n = int(want_send[d, f])
            assert s[d, f] == n
            np.testing.assert_array_equal(s[d, 2 + f * C_:2 + f * C_ + n], want_send[d, 2 + f * C_:2 + f * C_ + n])


def _run_ranks(steps):
    """Run fn(rank) on one thread per rank; re-raise the first failure."""
    errs = []

    def wrap(fn):
        try:
            fn()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=wrap, args=(fn,)) for fn in steps]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    if errs:
        raise errs[0]


def test_sharded_w1_equals_fused_single_gpu_step(device):
    """At W = 1 the sharded step (route, in-place exchange, gather, indexed T1, flat dedup, DP
    Adam) must reproduce the single-GPU fused step bit for bit."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep
    from two_tower_recommender_model_amd.sharded import FusedShardedTwoTowerStep, ThreadComm

    B, D, N = 2048, 128, [40_000, 60_000]
    ref_step = FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, device, seed=6)
    assert ref_step.gather and ref_step.dedup_single and ref_step.combined_bwd
    full = [ref_step.tables.table_view(f).cpu().clone() for f in range(2)]
    sh = FusedShardedTwoTowerStep(ThreadComm.group(1)[0], N, D, [128, 64], B, device, full_tables=full, seed=6)
    sh.params.copy_(ref_step.params)
    sh.towers.update(sh.params, do_adam=False)
    g = torch.Generator().manual_seed(2)
    for s in range(3):
        cols = [torch.randint(-n, 2 * n, (B,), generator=g) for n in N]
        cols[0][:40] = 0
        cols[1][40:90] = 777  # a hot row (> 14 lookups)
        lab = torch.randint(0, 2, (B,), generator=g).to(torch.int32)
        for st in (ref_step, sh):
            st.load_batch([c.to(device) for c in cols], lab.to(device))
            st.step()
    torch.cuda.synchronize()
    sh.check()
    for f in range(2):
        assert torch.equal(sh.tables.table_view(f), ref_step.tables.table_view(f))
        assert torch.equal(sh.tables.state_view(f), ref_step.tables.state_view(f))
    assert torch.equal(sh.params, ref_step.params)
    assert torch.equal(sh.logits, ref_step.logits)
    assert float(sh.loss) == float(ref_step.loss)


@pytest.mark.parametrize("W,sharding", [(2, ("row_wise", "row_wise")), (3, ("table_wise", "row_wise")),
                                        (4, ("row_wise", "table_wise")), (8, ("row_wise", "row_wise"))])
def test_sharded_threads_vs_oracle(device, W, sharding):
    from two_tower_recommender_model_amd.sharded import FusedShardedTwoTowerStep, ThreadComm

    B, D, N, lr = 1024, 64, [9_000, 12_345], 0.02
    gen = torch.Generator().manual_seed(W)
    full = [torch.empty(n, D).uniform_(-0.05, 0.05, generator=gen) for n in N]
    states = [torch.zeros(n) for n in N]
    comms = ThreadComm.group(W)
    steps = [None] * W

    def build(r):
        torch.cuda.set_device(device)
        steps[r] = FusedShardedTwoTowerStep(comms[r], N, D, [128, 64], B, device, sharding=sharding,
                                            tw_owners=[W - 1, 0], full_tables=full, lr_emb=lr, seed=3)

    _run_ranks([lambda r=r: build(r) for r in range(W)])
    for s in range(3):
        batches = []
        for r in range(W):
            cols = [torch.randint(0, 2 * n, (B,), generator=gen) for n in N]
            cols[0][torch.rand(B, generator=gen) < 0.05] = 0
            cols[1][:30] = 4242  # hot on one rank
            lab = torch.randint(0, 2, (B,), generator=gen).to(torch.int32)
            batches.append((cols, lab))
            steps[r].load_batch([c.to(device) for c in cols], lab.to(device))
        torch.cuda.synchronize()

        def run(r):
            torch.cuda.set_device(device)
            steps[r].step()
            torch.cuda.synchronize()

        _run_ranks([lambda r=r: run(r) for r in range(W)])
        # (a) every rank's tower inputs are the oracle rows (pre-update)
        rows_all, grads_all = [[] for _ in N], [[] for _ in N]
        for r in range(W):
            st = steps[r]
            st.check()
            pos = st.pos.cpu().numpy()
            rin = st.rows_in.cpu()
            gout = st.grad_out.cpu()
            cols, _ = batches[r]
            for f in range(2):
                p = pos[f * B:(f + 1) * B]
                kept = p >= 0
                ids = np.mod(cols[f].numpy()[kept], N[f])
                assert np.array_equal(kept, cols[f].numpy() != 0)
                got = rin[torch.from_numpy(p[kept]).long()]  # bf16 rows (the all-to-all carries bf16)
                want = full[f][torch.from_numpy(ids)].to(torch.bfloat16)
                if s == 0:  # initial tables: bit for bit (after the same bf16 rounding)
                    assert torch.equal(got, want), (r, f)
                else:  # updated rows: the row-wise mean of G^2 is reduced in another order -> one bf16 ulp
                    np.testing.assert_allclose(got.float().numpy(), want.float().numpy(), rtol=1e-2, atol=1e-7)
                rows_all[f].append(torch.from_numpy(ids))
                grads_all[f].append(gout[torch.from_numpy(p[kept]).long()])
        # (b) oracle update from the union of the gradient rows, rank-major
        for f in range(2):
            ref.rowwise_adagrad_from_lookups(full[f], states[f], torch.cat(rows_all[f]), torch.cat(grads_all[f]),
                                             lr, 1e-10)
        for r in range(W):
            st = steps[r]
            for f in range(2):
                n = st.local_rows[f]
                lo = st.row_lo[f]
                np.testing.assert_allclose(st.tables.table_view(f)[:n].cpu().numpy(), full[f][lo:lo + n].numpy(),
                                           rtol=1e-5, atol=1e-7)
                np.testing.assert_allclose(st.tables.state_view(f)[:n].cpu().numpy(), states[f][lo:lo + n].numpy(),
                                           rtol=1e-5, atol=1e-10)
        # (c) data-parallel towers identical everywhere
        for r in range(1, W):
            assert torch.equal(steps[r].params, steps[0].params)
    # every row held exactly once
    for f in range(2):
        assert sum(steps[r].local_rows[f] for r in range(W)) == N[f]


def test_sharded_overflow_raises(device):
    from two_tower_recommender_model_amd import _lib
    from two_tower_recommender_model_amd.sharded import FusedShardedTwoTowerStep, ThreadComm

    W, B, D, N = 2, 512, 64, [1000, 1000]
    comms = ThreadComm.group(W)
    steps = [None] * W

    def build(r):
        steps[r] = FusedShardedTwoTowerStep(comms[r], N, D, [128, 64], B, device, capacity=64, seed=1)

    _run_ranks([lambda r=r: build(r) for r in range(W)])
    for r in range(W):
        steps[r].load_batch([torch.full((B,), 7, device=device), torch.full((B,), 9, device=device)],
                            torch.zeros(B, dtype=torch.int32, device=device))
    _run_ranks([lambda r=r: steps[r].step() for r in range(W)])
    torch.cuda.synchronize()
    with pytest.raises(_lib.TTError, match="capacity"):
        steps[0].check()


@pytest.mark.parametrize("overlap", [False, True])
def test_sharded_rccl_world1_graph_equals_eager(device, overlap):
    """The production comm (torch.distributed "nccl" = RCCL) with its collectives captured into
    HIP graphs, at world size 1 with the collectives forced on: identical to eager ThreadComm. Run
    in a child process (a process group and RCCL-in-graph state stay out of this test process).
    overlap: the gradient all-to-all and tower all-reduce on RCCL's stream (overlap_comm=True)."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "rccl_graph_check.py")] + (["--overlap"] if overlap else []),
                       capture_output=True, text=True,
                       timeout=300, cwd=os.path.dirname(here))
    assert r.returncode == 0 and "RCCL-GRAPH-OK" in r.stdout, (r.returncode, r.stdout[-1500:], r.stderr[:3000],
                                                               r.stderr[-1500:])
