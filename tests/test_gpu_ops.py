"""Parity of every C-ABI kernel against the oracle on the GPU (``-m gpu``).

Tolerances: integer/index outputs bit-exact; fp32 embedding path rtol 1e-5 / atol 1e-6*max(1,L)
(summation order); bf16-MFMA tower GEMMs: vs the exact product of the bf16-rounded operands
|err| <= 2e-6 * (|A| @ |B|) + 1e-6 (fp32 accumulation), vs fp32 relative Frobenius error < 1e-2."""
import zlib

import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    from two_tower_recommender_model_amd import ops as _ops

    return _ops


@pytest.mark.parametrize("case", ["i32", "i64", "big", "allzero"])
def test_kjt_build_bit_exact_vs_reference_golden(ops, device, case):
    g = load_golden(f"kjt_{case}.npz")
    dt = torch.from_numpy(g["user_id"]).dtype
    cols = [torch.from_numpy(g["user_id"]).to(device), torch.from_numpy(g["product_id"]).to(device)]
    values, lengths, offsets, lpk = ops.kjt_build_mod_dropzero(cols, list(g["num_embeddings"]))
    torch.cuda.synchronize()
    n = int(offsets[-1])
    np.testing.assert_array_equal(lengths.cpu().numpy(), g["lengths"])
    np.testing.assert_array_equal(offsets.cpu().numpy(), g["offsets"])
    if g["values"].size:
        assert values.dtype == dt
        np.testing.assert_array_equal(values[:n].cpu().numpy(), g["values"])
    else:
        assert n == 0
    B = g["user_id"].size
    np.testing.assert_array_equal(lpk.cpu().numpy(), [g["lengths"][:B].sum(), g["lengths"][B:].sum()])


@pytest.mark.parametrize("n", [0, 1, 1023, 1024, 1025, 70000])
def test_complete_cumsum(ops, device, n):
    x = torch.randint(0, 5, (n,), dtype=torch.int32)
    out = ops.complete_cumsum(x.to(device)).cpu().numpy()
    np.testing.assert_array_equal(out, ref.complete_cumsum(x.numpy()))


def test_kjt_build_large_scan(ops, device):
    g = torch.Generator().manual_seed(3)
    B = 50000
    cols = [torch.randint(0, 5, (B,), generator=g, dtype=torch.int64) for _ in range(3)]
    N = [3, 7, 2**31 + 11]
    values, lengths, offsets, _ = ops.kjt_build_mod_dropzero([c.to(device) for c in cols], N)
    v, l, o = ref.kjt_build([c.numpy() for c in cols], N)
    np.testing.assert_array_equal(offsets.cpu().numpy(), o)
    np.testing.assert_array_equal(values[: o[-1]].cpu().numpy(), v)


@pytest.mark.parametrize("perm", [[2, 0, 1], [1, 1, 0, 2], [0]])
def test_kjt_permute(ops, device, perm):
    rng = np.random.default_rng(0)
    F_, B = 3, 33
    lengths = rng.integers(0, 5, F_ * B).astype(np.int32)
    values = rng.integers(0, 10**6, int(lengths.sum())).astype(np.int64)
    weights = rng.random(values.size).astype(np.float32)
    L = torch.from_numpy(lengths).to(device)
    O = ops.complete_cumsum(L)
    ol, oo, ov, ow = ops.kjt_permute(L, O, torch.from_numpy(values).to(device), F_, B, perm,
                                     weights=torch.from_numpy(weights).to(device))
    rl, rv, rw = ref.kjt_permute(lengths, values, F_, B, perm, weights)
    np.testing.assert_array_equal(ol.cpu().numpy(), rl)
    np.testing.assert_array_equal(oo.cpu().numpy(), ref.complete_cumsum(rl))
    np.testing.assert_array_equal(ov.cpu().numpy(), rv)
    np.testing.assert_array_equal(ow.cpu().numpy(), rw)


@pytest.mark.parametrize("W", [2, 8])
def test_block_bucketize(ops, device, W):
    rng = np.random.default_rng(W)
    F_, B = 3, 40
    N = [100, 1000, 7]
    lengths = rng.integers(0, 6, F_ * B).astype(np.int32)
    offs = ref.complete_cumsum(lengths)
    vals = []
    for i in range(F_ * B):
        vals.extend(rng.integers(0, N[i // B] + 3, lengths[i]).tolist())
    values = np.asarray(vals, np.int64)
    bs = [(n + W - 1) // W for n in N]
    L = torch.from_numpy(lengths).to(device)
    nl, no, nv = ops.block_bucketize(L, ops.complete_cumsum(L), torch.from_numpy(values).to(device), F_, B, bs, W)
    rl, rv = ref.block_bucketize(lengths, values, F_, B, bs, W)
    np.testing.assert_array_equal(nl.cpu().numpy(), rl)
    np.testing.assert_array_equal(no.cpu().numpy(), ref.complete_cumsum(rl))
    np.testing.assert_array_equal(nv.cpu().numpy(), rv)


def _make_kjt(rng, F_, B, rows, maxlen, zipf=False, dtype=np.int64):
    lengths = rng.integers(0 if maxlen > 1 else 1, maxlen + 1, F_ * B).astype(np.int32)
    vals = []
    for i in range(F_ * B):
        n = rows[i // B]
        if zipf:
            v = (rng.zipf(1.3, lengths[i]) - 1) % n
        else:
            v = rng.integers(0, n, lengths[i])
        vals.extend(v.tolist())
    return lengths, np.asarray(vals, dtype=dtype)


CASES = [
    # (name, T, feature_table, rows, dims, B, maxlen, zipf, dtype)
    ("d64_single", 2, [0, 1], [5000, 3000], [64, 64], 257, 1, False, np.int64),
    ("d128_single_i32", 2, [0, 1], [4000, 6000], [128, 128], 300, 1, False, np.int32),
    ("d16_multi", 2, [0, 1], [50, 80], [16, 16], 64, 20, False, np.int64),
    ("mixed_dims_shared", 3, [0, 1, 2, 0], [700, 300, 900], [36, 4, 128], 77, 7, True, np.int64),
    ("t16_d128", 16, list(range(16)), [2000] * 16, [128] * 16, 96, 1, False, np.int64),
    ("zipf_hot", 2, [0, 1], [100, 50], [128, 64], 512, 3, True, np.int64),
    ("odd_dim", 2, [0, 1], [100, 100], [3, 10], 50, 4, False, np.int64),
    ("d512", 1, [0], [300], [512], 40, 3, True, np.int64),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("pooling", ["sum", "mean"])
def test_pooled_fwd_and_fused_rowwise_adagrad(ops, device, case, pooling):
    name, T, ft, rows, dims, B, maxlen, zipf, dtype = case
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    F_ = len(ft)
    lengths, values = _make_kjt(rng, F_, B, [rows[t] for t in ft], maxlen, zipf, dtype)
    offsets = ref.complete_cumsum(lengths)
    ts = ops.TableSet(rows, dims, ft, device)
    ts.init_uniform_(torch.Generator(device=device).manual_seed(5))
    tables0 = [ts.table_view(t).cpu().clone() for t in range(T)]
    V = torch.from_numpy(values).to(device)
    O = torch.from_numpy(offsets).to(device)
    pool = 1 if pooling == "mean" else 0
    out = ts.pooled_fwd(V, O, B, pooling=pool)
    want = ref.pooled_fwd(tables0, ft, torch.from_numpy(values), torch.from_numpy(offsets), B, pooling)
    atol = 1e-6 * max(1, maxlen)
    np.testing.assert_allclose(out.cpu().numpy(), want.numpy(), rtol=1e-5, atol=atol)
    if maxlen == 1 and pooling == "sum":
        # single-hot sum pooling is a pure gather: bit-exact
        np.testing.assert_array_equal(out.cpu().numpy(), want.numpy())
    # backward with fused row-wise Adagrad, 2 steps
    lr, eps = 0.05, 1e-10
    tabs = [t.clone() for t in tables0]
    states = [torch.zeros(r) for r in rows]
    for step in range(2):
        gout = torch.randn(B, ts.out_dim, generator=torch.Generator().manual_seed(step))
        grads = ref.pooled_bwd_dense(tabs, ft, torch.from_numpy(values), torch.from_numpy(offsets), B, gout, pooling)
        for t in range(T):
            ref.rowwise_adagrad(tabs[t], states[t], grads[t], lr, eps)
        ts.bwd_prepare(V, O, B, max_lookups=max(1, values.size))
        ts.bwd_rowwise_adagrad(gout.to(device), O, B, lr, eps, pooling=pool)
    torch.cuda.synchronize()
    for t in range(T):
        np.testing.assert_allclose(ts.table_view(t).cpu().numpy(), tabs[t].numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(ts.state_view(t).cpu().numpy(), states[t].numpy(), rtol=1e-5, atol=1e-9)


def test_fused_adagrad_deterministic(ops, device):
    """Hot rows (up to ~2000 lookups of one row) included: every row's gradient is summed in
    ascending bag order, so repeated runs agree bit for bit (the scatter's order does not)."""
    rng = np.random.default_rng(7)
    B, rows = 2048, [64, 4096]
    lengths, values = _make_kjt(rng, 2, B, rows, 4, zipf=True)
    offsets = torch.from_numpy(ref.complete_cumsum(lengths)).to(device)
    V = torch.from_numpy(values).to(device)
    gout = torch.randn(B, 256, generator=torch.Generator().manual_seed(3)).to(device)
    results = []
    for _ in range(3):
        ts = ops.TableSet(rows, [128, 128], [0, 1], device)
        ts.init_uniform_(torch.Generator(device=device).manual_seed(1))
        ts.bwd_prepare(V, offsets, B, values.size)
        ts.bwd_rowwise_adagrad(gout, offsets, B, 0.1, 1e-10)
        results.append(ts.weights.clone())
    assert torch.equal(results[0], results[1]) and torch.equal(results[0], results[2])


@pytest.mark.parametrize("pooling", ["sum", "mean"])
def test_fused_adagrad_hot_rows(ops, device, pooling):
    """Rows looked up thousands of times per step (several LDS passes of the hot-row kernel) and a
    single bag holding one id 5000 times (the repeated-bag-id pass), narrow (D=128) and generic
    (D=256) tables, against the oracle; and bitwise equal to a second run."""
    rng = np.random.default_rng(11)
    B, rows, dims = 1024, [3, 40], [128, 256]
    lengths = rng.integers(0, 20, 2 * B).astype(np.int32)
    lengths[5] = 5000
    vals = []
    for i in range(2 * B):
        n = rows[i // B]
        vals.extend([1] * lengths[i] if i == 5 else rng.integers(0, n, lengths[i]).tolist())
    values = np.asarray(vals, np.int64)
    offsets = ref.complete_cumsum(lengths)
    pool = 1 if pooling == "mean" else 0
    gout = torch.randn(B, sum(dims), generator=torch.Generator().manual_seed(4))
    results = []
    for _ in range(2):
        ts = ops.TableSet(rows, dims, [0, 1], device)
        ts.init_uniform_(torch.Generator(device=device).manual_seed(2))
        tables0 = [ts.table_view(t).cpu().clone() for t in range(2)]
        V, O = torch.from_numpy(values).to(device), torch.from_numpy(offsets).to(device)
        ts.bwd_prepare(V, O, B, values.size)
        ts.bwd_rowwise_adagrad(gout.to(device), O, B, 0.05, 1e-10, pooling=pool)
        results.append(ts.weights.clone())
    assert torch.equal(results[0], results[1])
    grads = ref.pooled_bwd_dense(tables0, [0, 1], torch.from_numpy(values), torch.from_numpy(offsets), B, gout,
                                 pooling)
    states = [torch.zeros(r) for r in rows]
    for t in range(2):
        ref.rowwise_adagrad(tables0[t], states[t], grads[t], 0.05, 1e-10)
        np.testing.assert_allclose(ts.table_view(t).cpu().numpy(), tables0[t].numpy(), rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(ts.state_view(t).cpu().numpy(), states[t].numpy(), rtol=1e-4, atol=1e-9)


def test_pooled_bwd_dense(ops, device):
    rng = np.random.default_rng(9)
    B, rows, ft = 100, [300, 200], [0, 1, 1]
    lengths, values = _make_kjt(rng, 3, B, [rows[t] for t in ft], 5)
    offsets = ref.complete_cumsum(lengths)
    ts = ops.TableSet(rows, [32, 32], ft, device)
    ts.init_uniform_()
    gout = torch.randn(B, ts.out_dim)
    gw = torch.zeros_like(ts.weights)
    ts.bwd_dense(gout.to(device), torch.from_numpy(values).to(device), torch.from_numpy(offsets).to(device), B, gw)
    want = ref.pooled_bwd_dense([ts.table_view(t).cpu() for t in range(2)], ft, torch.from_numpy(values),
                                torch.from_numpy(offsets), B, gout)
    for t in range(2):
        o = ts.weight_offsets[t]
        got = gw[o:o + rows[t] * 32].view(rows[t], 32).cpu()
        np.testing.assert_allclose(got.numpy(), want[t].numpy(), rtol=1e-5, atol=1e-5)


def _bf16_gemm_check(got, a, b):
    """got ~= a @ b where the kernel rounds a and b to bf16 and accumulates in fp32: compare with
    the exact (fp64) product of the bf16-rounded operands to fp32-accumulation tolerance, and
    with the fp32 product to bf16 tolerance (relative Frobenius error <= 1e-2)."""
    ab = a.to(torch.bfloat16).double()
    bb = b.to(torch.bfloat16).double()
    exact = ab @ bb
    bound = (ab.abs() @ bb.abs()) * 2e-6 + 1e-6
    err = (got.double() - exact).abs()
    assert (err <= bound).all(), f"max err vs bf16-exact {err.max().item()}"
    fp32 = a.double() @ b.double()
    rel = (got.double() - fp32).norm() / (fp32.norm() + 1e-12)
    assert rel < 1e-2, f"relative error vs fp32 {rel.item()}"


@pytest.mark.parametrize("M,N,K,groups,xbf16", [(4096, 128, 64, 2, False), (1000, 64, 128, 1, False),
                                                 (513, 128, 1024, 2, False), (77, 5, 36, 1, True)])
def test_linear_fwd_bwd_vs_fp32(ops, device, M, N, K, groups, xbf16):
    g = torch.Generator(device="cpu").manual_seed(M + N)
    xs = [torch.randn(M, K, generator=g) for _ in range(groups)]
    ws = [torch.randn(N, K, generator=g) / K**0.5 for _ in range(groups)]
    bs = [torch.randn(N, generator=g) for _ in range(groups)]
    xd = [x.to(device).to(torch.bfloat16) if xbf16 else x.to(device) for x in xs]
    ys = ops.linear_fwd(xd, [w.to(device) for w in ws], [b.to(device) for b in bs], relu=True)
    for i in range(groups):
        xr = xd[i].float().cpu()
        pre = ys[i].cpu() > 0
        # pre-activation check on the positive part (relu(x) > 0 <=> x > 0)
        z = torch.where(pre, ys[i].cpu(), torch.zeros(()))
        want = torch.relu(xr.to(torch.bfloat16).double() @ ws[i].to(torch.bfloat16).double().T + bs[i].double())
        bound = (xr.to(torch.bfloat16).double().abs() @ ws[i].to(torch.bfloat16).double().abs().T) * 2e-6 + 1e-6
        assert ((z.double() - want).abs() <= bound).all()
    # backward
    dys = [torch.randn(M, N, generator=g) for _ in range(groups)]
    dxs = ops.linear_bwd_data([d.to(device) for d in dys], ys, [w.to(device) for w in ws], relu=True)
    dws, dbs = ops.linear_bwd_weight([d.to(device) for d in dys], ys, xd, relu=True)
    for i in range(groups):
        y = ys[i].cpu()
        dz = dys[i] * (y > 0)
        _bf16_gemm_check(dxs[i].cpu(), dz, ws[i])
        _bf16_gemm_check(dws[i].cpu(), dz.T.contiguous(), xd[i].float().cpu())
        np.testing.assert_allclose(dbs[i].cpu().numpy(), dz.sum(0).numpy(), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("B,dim,ldt", [(8192, 64, torch.int32), (2, 8, torch.int64), (1000, 33, torch.float32)])
def test_dot_bce(ops, device, B, dim, ldt):
    g = torch.Generator().manual_seed(B)
    q = torch.rand(B, dim, generator=g)
    c = torch.rand(B, dim, generator=g)
    y = torch.randint(0, 2, (B,), generator=g).to(ldt)
    qq = q.clone().requires_grad_(True)
    cc = c.clone().requires_grad_(True)
    logits, loss = ref.dot_bce(qq, cc, y)
    loss.backward()
    k = ops.DotBCE(device, B)
    dq = torch.empty(B, dim, device=device)
    dc = torch.empty(B, dim, device=device)
    for _ in range(2):  # second call checks the arrival counter was reset
        lg, ls = k(q.to(device), c.to(device), y.to(device), dq=dq, dc=dc)
    np.testing.assert_allclose(lg.cpu().numpy().reshape(-1), logits.detach().numpy().reshape(-1), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(float(ls), float(loss), rtol=1e-5)
    np.testing.assert_allclose(dq.cpu().numpy(), qq.grad.numpy(), rtol=1e-4, atol=1e-8)
    np.testing.assert_allclose(dc.cpu().numpy(), cc.grad.numpy(), rtol=1e-4, atol=1e-8)


def test_dot_bce_batch_of_one(ops, device):
    """B = 1: the op (like torch's BCEWithLogits on [1] logits) is defined; the reference's task
    squeezes the logits to 0-d (03_model_training.py:452) and BCEWithLogitsLoss then raises — the
    oracle restatement and the drop-in TwoTowerTrainTask raise the same ValueError."""
    g = torch.Generator().manual_seed(1)
    q, c = torch.rand(1, 8, generator=g), torch.rand(1, 8, generator=g)
    y = torch.ones(1, dtype=torch.int64)
    qq, cc = q.clone().requires_grad_(True), c.clone().requires_grad_(True)
    logits = (qq * cc).sum(1)  # not squeezed
    loss = torch.nn.BCEWithLogitsLoss()(logits, y.float())
    loss.backward()
    k = ops.DotBCE(device, 1)
    dq, dc = torch.empty(1, 8, device=device), torch.empty(1, 8, device=device)
    lg, ls = k(q.to(device), c.to(device), y.to(device), dq=dq, dc=dc)
    np.testing.assert_allclose(lg.cpu().numpy(), logits.detach().numpy(), rtol=1e-5)
    np.testing.assert_allclose(float(ls), float(loss), rtol=1e-5)
    np.testing.assert_allclose(dq.cpu().numpy(), qq.grad.numpy(), rtol=1e-4, atol=1e-8)
    with pytest.raises(ValueError, match="must be the same as input size"):
        ref.dot_bce(q, c, y)

    import two_tower_recommender_model_amd as tt

    tt.install_torchrec_alias()
    from torchrec.datasets.utils import Batch
    from torchrec.modules.embedding_configs import EmbeddingBagConfig
    from torchrec.modules.embedding_modules import EmbeddingBagCollection
    from torchrec.sparse.jagged_tensor import KeyedJaggedTensor

    from two_tower_recommender_model_amd.task import TwoTower, TwoTowerTrainTask

    ebc = EmbeddingBagCollection(tables=[EmbeddingBagConfig(name=f"t_{f}", embedding_dim=32, num_embeddings=10,
                                                            feature_names=[f]) for f in ("user_id", "product_id")],
                                 device=device)
    task = TwoTowerTrainTask(TwoTower(ebc, [32, 32], device=device))
    kjt = KeyedJaggedTensor.from_lengths_sync(["user_id", "product_id"], torch.tensor([3, 4], device=device),
                                              torch.ones(2, dtype=torch.int32, device=device))
    with pytest.raises(ValueError, match="must be the same as input size"):
        task(Batch(dense_features=torch.zeros(1), sparse_features=kjt,
                   labels=torch.ones(1, dtype=torch.int32, device=device)))


def test_adam(ops, device):
    g = torch.Generator().manual_seed(0)
    p = torch.randn(49536, generator=g)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    pd, md, vd = p.to(device), m.to(device), v.to(device)
    st = torch.zeros(2, dtype=torch.int64, device=device)
    for step in range(1, 4):
        grad = torch.randn(49536, generator=g)
        ref.adam([p], [grad], [m], [v], step, lr=0.01)
        ops.adam_step(pd, grad.to(device), md, vd, st, lr=0.01)
    np.testing.assert_allclose(pd.cpu().numpy(), p.numpy(), rtol=1e-5, atol=1e-6)
    assert int(st[0]) == 3 and int(st[1]) == 0


@pytest.mark.parametrize("M,N,K,groups", [(1000, 128, 64, 2), (300, 64, 128, 1), (129, 33, 1024, 2)])
def test_linear_fp32_parity_mode(ops, device, M, N, K, groups):
    """precision='fp32': exact fp32 operands on v_mfma_f32_16x16x4_f32 — matches the fp64 product
    to fp32 accumulation error (|err| <= 1e-5 * (|A| @ |B|) + 1e-6)."""
    g = torch.Generator().manual_seed(K)
    xs = [torch.randn(M, K, generator=g) for _ in range(groups)]
    ws = [torch.randn(N, K, generator=g) / K**0.5 for _ in range(groups)]
    bs = [torch.randn(N, generator=g) for _ in range(groups)]
    ys = ops.linear_fwd([x.to(device) for x in xs], [w.to(device) for w in ws], [b.to(device) for b in bs],
                        relu=True, precision="fp32")
    dys = [torch.randn(M, N, generator=g) for _ in range(groups)]
    dxs = ops.linear_bwd_data([d.to(device) for d in dys], ys, [w.to(device) for w in ws], relu=True, precision="fp32")
    dws, dbs = ops.linear_bwd_weight([d.to(device) for d in dys], ys, [x.to(device) for x in xs], relu=True,
                                     precision="fp32")

    def close(got, a, b, add=None):
        exact = a.double() @ b.double()
        if add is not None:
            exact = exact + add.double()
        bound = (a.double().abs() @ b.double().abs()) * 1e-5 + 1e-6
        assert ((got.double() - exact).abs() <= bound).all(), (got.double() - exact).abs().max()

    for i in range(groups):
        y = ys[i].cpu()
        pos = y > 0
        pre = xs[i].double() @ ws[i].double().T + bs[i].double()
        assert ((y.double() - torch.relu(pre)).abs() <= (xs[i].abs().double() @ ws[i].abs().double().T) * 1e-5 + 1e-5).all()
        dz = dys[i] * pos
        close(dxs[i].cpu(), dz, ws[i])
        close(dws[i].cpu(), dz.T.contiguous(), xs[i])


@pytest.mark.parametrize("rows,dim", [(1, 4), (3, 7), (5000, 128), (1 << 17, 64)])
def test_table_prefault_reads_only(ops, device, rows, dim):
    """TableSet.prefault (tt_table_prefault): one load per page of the weights and the state, the
    last partial page included; nothing of the tables changes and the sink stays 0."""
    ts = ops.TableSet([rows, 3], [dim, dim], [0, 1], device)
    ts.init_uniform_(torch.Generator(device=device).manual_seed(0))
    ts.state.uniform_()
    w0, s0 = ts.weights.clone(), ts.state.clone()
    for page in (4096, 4, 65536):
        ts.prefault(page)
    torch.cuda.synchronize()
    assert torch.equal(ts.weights, w0) and torch.equal(ts.state, s0)
    assert int(ts._sink[0]) == 0


def test_table_prefault_argument_errors(ops, device):
    from two_tower_recommender_model_amd import _lib

    lib = _lib.load()
    sink = torch.zeros(1, dtype=torch.int32, device=device)
    buf = torch.zeros(16, dtype=torch.float32, device=device)
    assert lib.tt_table_prefault(buf.data_ptr(), 64, 6, sink.data_ptr(), None) != 0
    assert lib.tt_table_prefault(buf.data_ptr(), 64, 4096, None, None) != 0
    assert lib.tt_table_prefault(None, 0, 4096, sink.data_ptr(), None) == 0


def test_table_alloc_large_tableset_matches_caching_allocator(ops, device):
    """TableSet buffers >= TABLE_ALLOC_MIN_BYTES come from tt_table_alloc (contiguous when the
    driver can); the same weights in caching-allocator memory give bit-identical pooled sums, and
    the memory is released with the last view (a second allocation of the same size succeeds)."""
    rows = ops.TABLE_ALLOC_MIN_BYTES // (128 * 4) + 1000
    for _ in range(2):
        ts = ops.TableSet([rows, 64], [128, 128], [0, 1], device)
        assert isinstance(ts.weights, torch.Tensor) and ts.weights.dtype == torch.float32
        assert ts.weights.numel() >= rows * 128 and float(ts.state.abs().sum()) == 0.0
        ts.init_uniform_(torch.Generator(device=device).manual_seed(3))
        ref_ts = ops.TableSet([rows, 64], [128, 128], [0, 1], device, weights=ts.weights.clone())
        g = torch.Generator(device=device).manual_seed(4)
        B = 512
        values = torch.cat([torch.randint(0, rows, (B,), device=device, generator=g),
                            torch.randint(0, 64, (B,), device=device, generator=g)])
        offsets = torch.arange(0, 2 * B + 1, dtype=torch.int32, device=device)
        a = ts.pooled_fwd(values, offsets, B)
        b = ref_ts.pooled_fwd(values, offsets, B)
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        del ts, ref_ts, a, b
        import gc
        gc.collect()
        assert len(ops._PENDING_FREE) >= 1  # the weights (the state is below the threshold), freed later
    ops.free_tables()
    assert not ops._PENDING_FREE
