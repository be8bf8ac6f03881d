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


def _threads_vs_oracle(device, W, N, Fq, sharding, tw_owners, B, D, lr, layers, nsteps=3, seed=0, small=True):
    """W ranks as threads of one process over ThreadComm, F = len(N) single-hot features (0 .. Fq-1
    query, the rest candidate). Per step, against the state read from the shards before it: (a) the
    rows each rank's towers read are the table rows its ids name (bf16, bit for bit); (b) each
    rank's gradient rows dX, logits and tower gradient (sent x 1/W) against the fp64 emulation of
    the bf16 towers on ITS OWN batch and mean loss, element-wise (tower_emul.check_towers; the loss
    scale TorchRec's sharded EBC gives: the sum over ranks of the per-rank mean-loss gradients);
    (c) every touched row against the oracle's row-wise Adagrad over the union of the EMULATED
    gradient rows (ascending (rank, bag) order), tolerance from their bounds; (d) the towers
    against the oracle's Adam fed the fixed-order sum of the ranks' tower gradients x 1/W (DDP's
    mean all-reduce), identical on every rank. ``small``: tables initialised from one CPU copy and
    every untouched row checked unchanged (off for BASELINE-size tables: each rank draws its own
    shard and only the touched rows are read back)."""
    from tower_emul import check_adagrad, check_towers, emulate_bounds, split_params

    from two_tower_recommender_model_amd.sharded import FusedShardedTwoTowerStep, ThreadComm

    F = len(N)
    gen = torch.Generator().manual_seed(100 * W + F + seed)
    full = [torch.empty(n, D).uniform_(-0.05, 0.05, generator=gen) for n in N] if small else None
    comms = ThreadComm.group(W)
    ranks = [None] * W

    def build(r):
        torch.cuda.set_device(device)
        ranks[r] = FusedShardedTwoTowerStep(comms[r], N, D, layers, B, device, sharding=sharding,
                                            tw_owners=tw_owners, full_tables=full, lr_emb=lr, seed=3,
                                            num_query_features=Fq)

    _run_ranks([lambda r=r: build(r) for r in range(W)])
    in_dims = ranks[0].in_dims
    P = ranks[0].towers.num_params
    m_ref, v_ref = [torch.zeros(P)], [torch.zeros(P)]

    def read_rows(f, u):
        """(weights, state) of global rows u (CPU, sorted) of table f, from the shards that hold them."""
        w = torch.empty(u.numel(), D)
        st_ = torch.empty(u.numel())
        for r in range(W):
            st = ranks[r]
            lo, n = st.row_lo[f], st.local_rows[f]
            sel = (u >= lo) & (u < lo + n)
            if bool(sel.any()):
                idx = (u[sel] - lo).to(device)
                w[sel] = st.tables.table_view(f)[idx].cpu()
                st_[sel] = st.tables.state_view(f)[idx].cpu()
        return w, st_

    def snapshot():
        return [[(st.tables.table_view(f)[:st.local_rows[f]].cpu().clone(),
                  st.tables.state_view(f)[:st.local_rows[f]].cpu().clone()) for f in range(F)] for st in ranks]

    for s in range(nsteps):
        batches = []
        params0 = ranks[0].params.cpu().clone()
        for r in range(W):
            cols = [torch.randint(0, 2 * n, (B,), generator=gen) for n in N]
            cols[0][torch.rand(B, generator=gen) < 0.05] = 0
            cols[F - 1][:30] = 4242 % N[F - 1] + N[F - 1]  # hot on one rank (and past N: id % N)
            lab = torch.randint(0, 2, (B,), generator=gen).to(torch.int32)
            batches.append((cols, lab))
            ranks[r].load_batch([c.to(device) for c in cols], lab.to(device))
        uniq = []
        for f in range(F):
            ids = torch.cat([c[f][c[f] != 0] for c, _ in batches])
            uniq.append(torch.unique(torch.remainder(ids, N[f])))
        before = [read_rows(f, uniq[f]) for f in range(F)]
        snap = snapshot() if small else None
        torch.cuda.synchronize()

        def run(r):
            torch.cuda.set_device(device)
            ranks[r].step()
            torch.cuda.synchronize()

        _run_ranks([lambda r=r: run(r) for r in range(W)])
        _run_ranks([lambda r=r: ranks[r].check() for r in range(W)])
        rows_all, dx_all, eb_all = [[] for _ in N], [[] for _ in N], [[] for _ in N]
        tower_sum = torch.zeros(P)
        for r in range(W):
            st = ranks[r]
            cols, lab = batches[r]
            rin = st.rows_for(0).cpu()     # [F*B, D] bf16 rows T1 read
            gout = st.grad_rows(0).cpu()   # [F*B, D] the dX rows it sent
            pos = st.pos_in[0].cpu().numpy()
            keep = []
            for f in range(F):
                kept = pos[f * B:(f + 1) * B] >= 0
                assert np.array_equal(kept, cols[f].numpy() != 0)
                keep.append(kept)
                ids = torch.remainder(cols[f][torch.from_numpy(kept)], N[f])
                got = rin[f * B:(f + 1) * B][torch.from_numpy(kept)]
                want = before[f][0][torch.searchsorted(uniq[f], ids)].to(torch.bfloat16)
                assert torch.equal(got, want), (r, f)  # (a) bit for bit (the same bf16 rounding)
                rows_all[f].append(ids)
            # (b) this rank's logits, dX and tower gradient vs the emulation on its own batch
            x = rin.float()
            xq = torch.cat([x[f * B:(f + 1) * B] for f in range(Fq)], 1)
            xc = torch.cat([x[f * B:(f + 1) * B] for f in range(Fq, F)], 1)
            prm = split_params(params0, in_dims, layers)
            lg, loss, dxs, gw, amb = emulate_bounds(xq, xc, prm, layers, lab)
            dx_f, eb_f = [], []
            for f in range(F):
                t, j = (0, f) if f < Fq else (1, f - Fq)
                m = torch.from_numpy(keep[f]).double()[:, None]  # dropped lookups send no row
                dx_f.append(dxs[t][0][:, j * D:(j + 1) * D] * m)
                eb_f.append(dxs[t][1][:, j * D:(j + 1) * D] * m)
            dxs2 = [(torch.cat(dx_f[:Fq], 1), torch.cat(eb_f[:Fq], 1)),
                    (torch.cat(dx_f[Fq:], 1), torch.cat(eb_f[Fq:], 1))]
            got_dx = [torch.cat([gout[f * B:(f + 1) * B] for f in range(Fq)], 1),
                      torch.cat([gout[f * B:(f + 1) * B] for f in range(Fq, F)], 1)]
            sent = st.tower_grad_sent().cpu()
            glist, o = [], 0
            for p_ in prm:
                glist.append(sent[o:o + p_.numel()].reshape(p_.shape) * W)
                o += p_.numel()
            check_towers((lg, loss, dxs2, gw, amb), st.logits.cpu(), got_dx, glist, f"rank {r}")
            for f in range(F):
                k = torch.from_numpy(keep[f])
                dx_all[f].append(dx_f[f][k])
                eb_all[f].append(eb_f[f][k])
            tower_sum += sent  # fixed rank order, as the receivers sum
        # (c) every touched row vs the oracle fed the union of the emulated gradient rows, rank-major
        for f in range(F):
            inv = torch.searchsorted(uniq[f], torch.cat(rows_all[f]))
            w_got, s_got = read_rows(f, uniq[f])
            check_adagrad(w_got, s_got, before[f][0], before[f][1], inv, torch.cat(dx_all[f]), torch.cat(eb_all[f]),
                          lr, 1e-10, f"feature {f}")
        if small:  # untouched rows never move
            for r in range(W):
                st = ranks[r]
                for f in range(F):
                    lo, n = st.row_lo[f], st.local_rows[f]
                    untouched = torch.ones(n, dtype=torch.bool)
                    u = uniq[f]
                    untouched[(u[(u >= lo) & (u < lo + n)] - lo)] = False
                    w0, s0 = snap[r][f]
                    assert torch.equal(st.tables.table_view(f)[:n].cpu()[untouched], w0[untouched])
                    assert torch.equal(st.tables.state_view(f)[:n].cpu()[untouched], s0[untouched])
        # (d) Adam on the summed (mean) tower gradient; identical replicas
        p_ref = [params0.clone()]
        ref.adam(p_ref, [tower_sum], m_ref, v_ref, s + 1, 0.01)
        np.testing.assert_allclose(ranks[0].params.cpu().numpy(), p_ref[0].numpy(), rtol=1e-5, atol=1e-7)
        for r in range(1, W):
            assert torch.equal(ranks[r].params, ranks[0].params)
    # every row held exactly once
    for f in range(F):
        assert sum(ranks[r].local_rows[f] for r in range(W)) == N[f]
    return ranks


@pytest.mark.parametrize("W,sharding", [(2, ("row_wise", "row_wise")), (3, ("table_wise", "row_wise")),
                                        (4, ("row_wise", "table_wise")), (8, ("row_wise", "row_wise")),
                                        (2, ("table_wise", "table_wise")), (4, ("table_wise", "table_wise"))])
def test_sharded_threads_vs_oracle(device, W, sharding):
    """The reference's two features (user / item towers), W ranks as threads (_threads_vs_oracle)."""
    _threads_vs_oracle(device, W, [9_000, 12_345], 1, list(sharding), [W - 1, 0], 1024, 64, 0.02, [128, 64])


@pytest.mark.parametrize("W,F,Fq,plan", [(1, 4, 2, "rw"), (2, 6, 3, "mix"), (3, 4, 2, "tw"), (8, 16, 8, "tw"),
                                         (4, 2, 1, "config4")])
def test_sharded_multifeature_threads_vs_oracle(device, W, F, Fq, plan):
    """Several single-hot features per tower through the general T1 (BASELINE config 3's shape at
    small table sizes: 8 table-wise features per tower at W = 8; config 4's plan: the item table
    row-wise, the user table table-wise), W ranks as threads (_threads_vs_oracle)."""
    N = [5_000 + 1_000 * f for f in range(F)]
    if plan == "rw":
        sharding, owners = ["row_wise"] * F, [0] * F
    elif plan == "tw":
        sharding, owners = ["table_wise"] * F, [(f * 5) % W for f in range(F)]
    elif plan == "config4":
        sharding, owners = ["table_wise", "row_wise"], [W - 1, 0]
    else:
        sharding = ["row_wise" if f % 2 else "table_wise" for f in range(F)]
        owners = [f % W for f in range(F)]
    layers = [128, 64] if F * 32 <= 1024 else [64, 32]
    _threads_vs_oracle(device, W, N, Fq, sharding, owners, 512, 32 if F > 8 else 64, 0.02, layers, nsteps=2, seed=F)


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
    from child_util import run_child

    run_child(["tests/rccl_graph_check.py"], "RCCL-GRAPH-OK", timeout=300)


def test_sharded_pipeline_state_resets(device):
    """The pipelined state after a refused capture (the bench's eager fallback) and after a mid-run
    load_state_dict: both equal a clean eager run bit for bit (tests/sharded_pipeline_state_check.py,
    a child process over a one-rank RCCL group)."""
    from child_util import run_child

    run_child(["tests/sharded_pipeline_state_check.py"], "PIPELINE-STATE-OK", timeout=300)


def test_sharded_config3_w8_baseline_size(device):
    """BASELINE config 3 at its size on one MI355X: 8 ranks as threads, 16 single-hot tables (user_id
    50M, product_id 100M, 14 x 1M rows; 84 GB of fp32 tables), 8 features per tower, D 128, B 8192
    per rank, bf16 towers over 1024-wide inputs, every table table-wise (bench.tw_plan: two tables
    per rank) — against the oracle on the touched rows (_threads_vs_oracle, 2 steps)."""
    import bench

    N = bench.SHARDED["config3"]["N"]
    W = 8
    owners = bench.tw_plan(N, W)
    ranks = _threads_vs_oracle(device, W, N, 8, ["table_wise"] * len(N), owners, 8192, 128, 0.01, [128, 64],
                               nsteps=2, seed=33, small=False)
    assert ranks[0].in_dims == [1024, 1024]
    del ranks
    import gc

    gc.collect()
    torch.cuda.empty_cache()
