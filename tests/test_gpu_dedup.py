"""Two-launch single-hot dedup + fused row-wise Adagrad (csrc/dedup.hip) against the oracle
(dense index_add gradient + torchrec RowWiseAdagrad, oracle/ref.py) and against the KJT-form
kernels (tt_bwd_prepare_cols + tt_bwd_rowwise_adagrad). Rows with <= 14 lookups are summed in
ascending lookup order (the oracle's order); hot rows use a fixed 8-way interleave (tolerance)."""
import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    from two_tower_recommender_model_amd import ops as _ops

    return _ops


def _cols(N, B, zipf, seed, dtype=torch.int64, zero_frac=0.05):
    g = torch.Generator().manual_seed(seed)
    cols = []
    for n in N:
        if zipf:
            r = torch.floor(torch.exp(torch.rand(B, generator=g, dtype=torch.float64) * np.log(n))).to(torch.int64)
            x = (r * 2654435761) % n
        else:
            x = torch.randint(-n, 3 * n, (B,), generator=g)
        x[torch.rand(B, generator=g) < zero_frac] = 0
        cols.append(x.to(dtype))
    return cols


def _oracle_step(tables, states, cols, N, gout, lr, eps):
    B = cols[0].numel()
    v, _, o = ref.kjt_build([c.numpy() for c in cols], N)
    grads = ref.pooled_bwd_dense(tables, list(range(len(N))), torch.from_numpy(v).to(torch.int64),
                                 torch.from_numpy(o), B, gout)
    for t in range(len(N)):
        touched = torch.unique(torch.from_numpy(v[o[t * B]:o[(t + 1) * B]]).to(torch.int64))
        ref.rowwise_adagrad_sparse(tables[t], states[t], touched, grads[t][touched], lr, eps)


def _counts(cols, N):
    out = []
    for c, n in zip(cols, N):
        c = c.numpy()
        k = np.mod(c[c != 0], n)
        out.append(np.bincount(k, minlength=n))
    return out


@pytest.mark.parametrize("B,dims,zipf", [(4096, [128, 128], False), (8192, [64, 64], True),
                                         (3000, [32, 128], True), (1000, [128, 64], False)])
def test_dedup_cols_vs_oracle(ops, device, B, dims, zipf):
    N = [20000, 3000] if not zipf else [50000, 9000]
    lr, eps = 0.05, 1e-10
    ts = ops.TableSet(N, dims, [0, 1], device)
    ts.init_uniform_(torch.Generator(device=device).manual_seed(1))
    tables = [ts.table_view(t).cpu().clone() for t in range(2)]
    states = [torch.zeros(n) for n in N]
    for step in range(3):
        cols = _cols(N, B, zipf, seed=10 * step + B)
        gout = torch.randn(B, sum(dims), generator=torch.Generator().manual_seed(step))
        ts.dedup_insert_cols([c.to(device) for c in cols], N)
        ts.dedup_rowwise_adagrad(gout.to(device), B, lr, eps)
        _oracle_step(tables, states, cols, N, gout, lr, eps)
    torch.cuda.synchronize()
    for t in range(2):
        got_w, got_s = ts.table_view(t).cpu(), ts.state_view(t).cpu()
        np.testing.assert_allclose(got_s.numpy(), states[t].numpy(), rtol=1e-4, atol=1e-9)
        np.testing.assert_allclose(got_w.numpy(), tables[t].numpy(), rtol=1e-4, atol=1e-6)
    _assert_clean(ts)


def _assert_clean(ts):
    """After every update the workspace is clean: every slot free, hot-row counters zero, no
    deferred insert pending (dedup.hip dedup_layout: slots, keys, hot list, counters, claims,
    overflow entries)."""
    L = ts._dd_cap
    cap = 1024
    while cap < 16 * L:
        cap <<= 1
    al = lambda x: (x + 255) // 256 * 256  # noqa: E731
    sl = ts._dd_ws[:cap * 128].view(torch.int64).view(cap, 16).cpu()  # 128-B slots
    assert bool((sl[:, 0] == -1).all())
    o = cap * 128 + al(8 * L) + al(4 * (L // 31 + 1))
    assert ts._dd_ws[o:o + 16].view(torch.int32).cpu().tolist() == [0, 0, 0, 0]
    o_ovf = o + 256 + al(4 * L)
    G = (L + 63) // 64
    ovf = ts._dd_ws[o_ovf:o_ovf + 16 * 64 * G].view(torch.int64).view(G * 64, 2).cpu()
    assert bool((ovf[:, 0] == -1).all())


def test_dedup_cols_equals_kjt_path_when_not_hot(ops, device):
    """<= 14 lookups per row: the same ascending order as the KJT-form narrow kernel -> bitwise."""
    B, N, dims = 8192, [50_000, 80_000], [128, 128]
    cols = _cols(N, B, False, seed=5)
    cnt = _counts(cols, N)
    assert max(int(c.max()) for c in cnt) <= 14
    a = ops.TableSet(N, dims, [0, 1], device)
    a.init_uniform_(torch.Generator(device=device).manual_seed(2))
    b = ops.TableSet(N, dims, [0, 1], device)
    b.weights.copy_(a.weights)
    dcols = [c.to(device) for c in cols]
    for step in range(2):
        gout = torch.randn(B, 256, generator=torch.Generator().manual_seed(step)).to(device)
        a.dedup_insert_cols(dcols, N)
        a.dedup_rowwise_adagrad(gout, B, 0.05, 1e-10)
        b.bwd_prepare_cols(dcols, N)
        b.bwd_rowwise_adagrad(gout, None, B, 0.05, 1e-10)
    torch.cuda.synchronize()
    assert torch.equal(a.weights, b.weights)
    assert torch.equal(a.state, b.state)


def test_dedup_hot_rows_bitwise_reproducible(ops, device):
    """Heavy skew (rows with thousands of lookups): two identical runs give identical bits."""
    B, N, dims = 8192, [1000, 64], [128, 128]
    cols = _cols(N, B, True, seed=7, zero_frac=0.0)
    assert max(int(c.max()) for c in _counts(cols, N)) > 1000
    gout = torch.randn(B, 256, generator=torch.Generator().manual_seed(0)).to(device)
    res = []
    for _ in range(2):
        ts = ops.TableSet(N, dims, [0, 1], device)
        ts.init_uniform_(torch.Generator(device=device).manual_seed(3))
        for _ in range(2):
            ts.dedup_insert_cols([c.to(device) for c in cols], N)
            ts.dedup_rowwise_adagrad(gout, B, 0.05, 1e-10)
        torch.cuda.synchronize()
        res.append((ts.weights.clone(), ts.state.clone()))
        _assert_clean(ts)
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def test_dedup_all_dropped(ops, device):
    B, N = 512, [100, 100]
    ts = ops.TableSet(N, [64, 64], [0, 1], device)
    ts.init_uniform_(torch.Generator(device=device).manual_seed(0))
    w0 = ts.weights.clone()
    cols = [torch.zeros(B, dtype=torch.int64, device=device) for _ in N]
    ts.dedup_insert_cols(cols, N)
    ts.dedup_rowwise_adagrad(torch.ones(B, 128, device=device), B, 0.1, 1e-10)
    torch.cuda.synchronize()
    assert torch.equal(ts.weights, w0) and int(torch.count_nonzero(ts.state)) == 0


@pytest.mark.parametrize("zipf", [False, True])
def test_dedup_segments_vs_oracle(ops, device, zipf):
    """Sharded owner side: W*T segments of capacity C, keys = table << 40 | local row, grad row i."""
    rows, D, nseg, C = [7000, 3000], 128, 8, 700
    g = torch.Generator().manual_seed(11 + zipf)
    counts = torch.randint(0, C + 1, (nseg,), generator=g).to(torch.int32)
    keys = torch.full((nseg * C,), -1, dtype=torch.int64)
    for s in range(nseg):
        t = s % 2
        n = int(counts[s])
        if zipf:
            r = (torch.floor(torch.exp(torch.rand(n, generator=g, dtype=torch.float64) * np.log(rows[t])))
                 .to(torch.int64) * 40503) % rows[t]
        else:
            r = torch.randint(0, rows[t], (n,), generator=g)
        keys[s * C:s * C + n] = (t << 40) | r
    grad = torch.randn(nseg * C, D, generator=g)
    ts = ops.TableSet(rows, [D, D], [0, 1], device)
    ts.init_uniform_(torch.Generator(device=device).manual_seed(5))
    tables = [ts.table_view(t).cpu().clone() for t in range(2)]
    states = [torch.zeros(r) for r in rows]
    for step in range(2):
        ts.dedup_insert_segments(keys.to(device), counts.to(device), C)
        ts.dedup_rowwise_adagrad(grad.to(device), nseg * C, 0.02, 1e-10, flat=True)
        for t in range(2):
            gd = torch.zeros(rows[t], D)
            for s in range(nseg):
                n = int(counts[s])
                k = keys[s * C:s * C + n]
                sel = (k >> 40) == t
                gd.index_add_(0, k[sel] & ((1 << 40) - 1), grad[s * C:s * C + n][sel])
            touched = torch.nonzero(gd.abs().sum(1) > 0).flatten()
            ref.rowwise_adagrad_sparse(tables[t], states[t], touched, gd[touched], 0.02, 1e-10)
    torch.cuda.synchronize()
    for t in range(2):
        np.testing.assert_allclose(ts.state_view(t).cpu().numpy(), states[t].numpy(), rtol=1e-4, atol=1e-9)
        np.testing.assert_allclose(ts.table_view(t).cpu().numpy(), tables[t].numpy(), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("ids", ["uniform", "hot"])
def test_fused_step_single_stream_combined_equals_streams(device, ids):
    """The one-stream step (T1 with the dedup insert -> [T2 + row-wise Adagrad] -> T3) equals the
    side-stream variant and, for rows with <= 14 lookups, the KJT-form dedup, bit for bit."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    B, D, N = 2048, 128, [30000, 50000]
    kw = dict(seed=4, materialize_pooled=True)
    steps = [FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, device, combined_bwd=True, **kw),
             FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, device, combined_bwd=False, **kw),
             FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, device, dedup="kjt", **kw)]
    assert steps[0].gather and steps[0].dedup_single and not steps[2].dedup_single
    g = torch.Generator().manual_seed(3)
    for s in range(3):
        if ids == "uniform":
            cols = [torch.randint(0, 2 * n, (B,), generator=g) for n in N]
        else:
            cols = [torch.randint(1, 40, (B,), generator=g) * 101 for n in N]
        lab = torch.randint(0, 2, (B,), generator=g).to(torch.int32)
        for st in steps:
            st.load_batch([c.to(device) for c in cols], lab.to(device))
            st.step()
    torch.cuda.synchronize()
    a, b, c = steps
    for x, y in ((a, b),) + (((a, c),) if ids == "uniform" else ()):
        assert torch.equal(x.tables.weights, y.tables.weights)
        assert torch.equal(x.tables.state, y.tables.state)
        assert torch.equal(x.params, y.params)
        assert float(x.loss) == float(y.loss)
    _assert_clean(a.tables)
