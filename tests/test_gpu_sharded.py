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
                                        (4, ("row_wise", "table_wise")), (8, ("row_wise", "row_wise")),
                                        (2, ("table_wise", "table_wise")), (4, ("table_wise", "table_wise"))])
def test_sharded_threads_vs_oracle(device, W, sharding):
    """W ranks as threads: (a) the rows each rank's towers read are the oracle tables' rows; (b) each
    rank's gradient rows dX and its tower gradient (sent x 1/W) match the fp64 emulation of the bf16
    towers on ITS OWN batch and mean loss (the loss scale TorchRec's sharded EBC gives: the sum over
    ranks of the per-rank mean-loss gradients); (c) every shard equals the oracle's row-wise Adagrad
    over the union of the kernels' gradient rows (ascending (rank, bag) order); (d) the towers equal
    the oracle's Adam fed the fixed-order sum of the ranks' tower gradients x 1/W (DDP's mean
    all-reduce) and are identical on every rank."""
    from tower_emul import check_towers, emulate_bounds, split_params

    from two_tower_recommender_model_amd.sharded import FusedShardedTwoTowerStep, ThreadComm

    B, D, N, lr, layers = 1024, 64, [9_000, 12_345], 0.02, [128, 64]
    gen = torch.Generator().manual_seed(W)
    full = [torch.empty(n, D).uniform_(-0.05, 0.05, generator=gen) for n in N]
    states = [torch.zeros(n) for n in N]
    comms = ThreadComm.group(W)
    steps = [None] * W

    def build(r):
        torch.cuda.set_device(device)
        steps[r] = FusedShardedTwoTowerStep(comms[r], N, D, layers, B, device, sharding=sharding,
                                            tw_owners=[W - 1, 0], full_tables=full, lr_emb=lr, seed=3)

    _run_ranks([lambda r=r: build(r) for r in range(W)])
    P = steps[0].towers.num_params
    m_ref, v_ref = [torch.zeros(P)], [torch.zeros(P)]
    for s in range(3):
        batches = []
        params0 = steps[0].params.cpu().clone()
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
        _run_ranks([lambda r=r: steps[r].check() for r in range(W)])
        rows_all, grads_all = [[] for _ in N], [[] for _ in N]
        tower_sum = torch.zeros(P)
        for r in range(W):
            st = steps[r]
            cols, lab = batches[r]
            rin = st.rows_for(0).cpu()     # [F*B, D] bf16 rows T1 read
            gout = st.grad_rows(0).cpu()   # [F*B, D] the dX rows it sent
            pos = st.pos_in[0].cpu().numpy()
            for f in range(2):
                kept = pos[f * B:(f + 1) * B] >= 0
                assert np.array_equal(kept, cols[f].numpy() != 0)
                ids = np.mod(cols[f].numpy()[kept], N[f])
                got = rin[f * B:(f + 1) * B][torch.from_numpy(kept)]
                want = full[f][torch.from_numpy(ids)].to(torch.bfloat16)
                # (a) initial tables: bit for bit (after the same bf16 rounding); updated rows: the
                # row-wise mean of G^2 is reduced in another order -> one bf16 ulp
                if s == 0:
                    assert torch.equal(got, want), (r, f)
                else:
                    np.testing.assert_allclose(got.float().numpy(), want.float().numpy(), rtol=1e-2, atol=1e-7)
                rows_all[f].append(torch.from_numpy(ids))
                grads_all[f].append(gout[f * B:(f + 1) * B][torch.from_numpy(kept)])
            # (b) this rank's dX and tower gradient vs the emulation on its own batch
            x = rin.float()
            prm = split_params(params0, [D, D], layers)
            lg, loss, dxs, gw, amb = emulate_bounds(x[:B], x[B:], prm, layers, lab)
            keepm = [(cols[f] != 0).double()[:, None] for f in range(2)]  # dropped lookups send no row
            dxs = [(dxs[f][0] * keepm[f], dxs[f][1] * keepm[f]) for f in range(2)]
            sent = st.tower_grad_sent().cpu()
            glist, o = [], 0
            for p in prm:
                glist.append(sent[o:o + p.numel()].reshape(p.shape) * W)
                o += p.numel()
            check_towers((lg, loss, dxs, gw, amb), st.logits.cpu(), [gout[:B], gout[B:]], glist, f"rank {r}")
            tower_sum += sent  # fixed rank order, as the receivers sum
        # (c) oracle update from the union of the gradient rows, rank-major
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
        # (d) Adam on the summed (mean) tower gradient; identical replicas
        p_ref = [params0.clone()]
        ref.adam(p_ref, [tower_sum], m_ref, v_ref, s + 1, 0.01)
        np.testing.assert_allclose(steps[0].params.cpu().numpy(), p_ref[0].numpy(), rtol=1e-5, atol=1e-7)
        for r in range(1, W):
            assert torch.equal(steps[r].params, steps[0].params)
    # every row held exactly once
    for f in range(2):
        assert sum(steps[r].local_rows[f] for r in range(W)) == N[f]


@pytest.mark.parametrize("W", [2, 3])
def test_sharded_pipelined_equals_synchronous(device, W):
    """The pipelined schedule (two exchanges per step: the next batch's ids travel with this batch's
    gradients) gives bit for bit the results of the synchronous step, over a cyclic batch pool."""
    from two_tower_recommender_model_amd.sharded import FusedShardedTwoTowerStep, ThreadComm

    B, D, N = 512, 128, [7_000, 11_000]
    gen = torch.Generator().manual_seed(40 + W)
    full = [torch.empty(n, D).uniform_(-0.05, 0.05, generator=gen) for n in N]
    pools = []
    for r in range(W):
        pool = []
        for _ in range(4):
            cols = [torch.randint(0, 2 * n, (B,), generator=gen).to(device) for n in N]
            cols[1][:20] = 77  # a hot row
            pool.append((cols, torch.randint(0, 2, (B,), generator=gen).to(torch.int32).to(device)))
        pools.append(pool)
    runs = {}
    for mode in ("sync", "pipe"):
        comms = ThreadComm.group(W)
        steps = [None] * W

        def build(r):
            torch.cuda.set_device(device)
            steps[r] = FusedShardedTwoTowerStep(comms[r], N, D, [128, 64], B, device, full_tables=full, seed=8,
                                                sharding=("row_wise", "table_wise"), tw_owners=[0, W - 1])

        _run_ranks([lambda r=r: build(r) for r in range(W)])

        def go(r):
            torch.cuda.set_device(device)
            st = steps[r]
            if mode == "sync":
                for i in range(6):
                    st.load_batch(*pools[r][i % 4])
                    st.step()
            else:
                st.run_eager(pools[r], 6)
            torch.cuda.synchronize()

        _run_ranks([lambda r=r: go(r) for r in range(W)])
        runs[mode] = steps
    for r in range(W):
        a, b = runs["sync"][r], runs["pipe"][r]
        assert torch.equal(a.tables.weights, b.tables.weights)
        assert torch.equal(a.tables.state, b.tables.state)
        assert torch.equal(a.params, b.params) and torch.equal(a.exp_avg_sq, b.exp_avg_sq)
        assert float(a.loss) == float(b.loss)


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
        # rank 0 overflows (every id owned by rank 0), rank 1 does not: both must raise
        ids = 7 if r == 0 else 999
        steps[r].load_batch([torch.full((B,), ids, device=device), torch.full((B,), ids, device=device)],
                            torch.zeros(B, dtype=torch.int32, device=device))
    _run_ranks([lambda r=r: steps[r].step() for r in range(W)])
    torch.cuda.synchronize()
    raised = [False] * W

    def chk(r):
        try:
            steps[r].check()
        except _lib.TTError as e:
            assert "capacity" in str(e)
            raised[r] = True

    _run_ranks([lambda r=r: chk(r) for r in range(W)])
    assert all(raised)


def test_sharded_optimizer_state_resume(device):
    """gathered_state_dict(optimizer=True) + load_state_dict resumes bit-exactly (tables, row-wise
    Adagrad state, towers and their Adam moments / step), also across a different rank count."""
    from two_tower_recommender_model_amd.sharded import FusedShardedTwoTowerStep, ThreadComm

    B, D, N = 256, 64, [3_000, 5_000]
    gen = torch.Generator().manual_seed(5)
    batches = [([torch.randint(0, 2 * n, (B,), generator=gen).to(device) for n in N],
                torch.randint(0, 2, (B,), generator=gen).to(torch.int32).to(device)) for _ in range(4)]

    def make(W, seed):
        comms = ThreadComm.group(W)
        steps = [None] * W

        def build(r):
            torch.cuda.set_device(device)
            steps[r] = FusedShardedTwoTowerStep(comms[r], N, D, [128, 64], B, device, seed=seed)

        _run_ranks([lambda r=r: build(r) for r in range(W)])
        return steps

    def train(steps, bs):
        def go(r):
            torch.cuda.set_device(device)
            for cols, lab in bs:
                steps[r].load_batch(cols, lab)  # every rank the same batch (the check is resume only)
                steps[r].step()
            torch.cuda.synchronize()

        _run_ranks([lambda r=r: go(r) for r in range(len(steps))])

    def gathered(steps):
        out = {}

        def g(r):
            out[r] = steps[r].gathered_state_dict(optimizer=True)

        _run_ranks([lambda r=r: g(r) for r in range(len(steps))])
        return out[0]

    # 1 rank: 4 steps straight vs 2 steps, save, load into a fresh 1-rank step, 2 more
    a = make(1, 1)
    train(a, batches)
    b = make(1, 1)
    train(b, batches[:2])
    sd = gathered(b)
    c = make(1, 9)
    c[0].load_state_dict(sd)
    train(c, batches[2:])
    assert torch.equal(a[0].tables.weights, c[0].tables.weights)
    assert torch.equal(a[0].tables.state, c[0].tables.state)
    assert torch.equal(a[0].params, c[0].params) and torch.equal(a[0].exp_avg, c[0].exp_avg)
    # the state dict re-shards: 2 ranks take their rows of tables and Adagrad state
    d = make(2, 9)
    _run_ranks([lambda r=r: d[r].load_state_dict(sd) for r in range(2)])
    for r in range(2):
        for f, name in enumerate(("user_id", "product_id")):
            lo, n = d[r].spans(f)[r]
            assert torch.equal(d[r].tables.state_view(f)[:n].cpu(),
                               sd[f"optim.ebc.t_{name}.rowwise_adagrad_state"][lo:lo + n].cpu())
        assert int(d[r].adam_state[0]) == 2


def test_sharded_rccl_world1_graph_equals_eager(device):
    """The production comm (torch.distributed "nccl" = RCCL) with its collectives captured into
    pipelined HIP graphs, at world size 1 with the collectives forced on: identical to eager
    synchronous steps over ThreadComm. Run in a child process (a process group and RCCL-in-graph
    state stay out of this test process)."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "rccl_graph_check.py")], capture_output=True, text=True,
                       timeout=300, cwd=os.path.dirname(here))
    assert r.returncode == 0 and "RCCL-GRAPH-OK" in r.stdout, (r.returncode, r.stdout[-1500:], r.stderr[:3000],
                                                               r.stderr[-1500:])


def test_sharded_pipeline_state_resets(device):
    """The pipelined state after a refused capture (the bench's eager fallback) and after a mid-run
    load_state_dict: both equal a clean eager run bit for bit (tests/sharded_pipeline_state_check.py,
    a child process over a one-rank RCCL group)."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "sharded_pipeline_state_check.py")], capture_output=True,
                       text=True, timeout=300, cwd=os.path.dirname(here))
    assert r.returncode == 0 and "PIPELINE-STATE-OK" in r.stdout, (r.returncode, r.stdout[-1500:], r.stderr[-3000:])
