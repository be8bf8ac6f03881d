"""Parity of the PRODUCTION step at the BASELINE.json sizes.

The step under test is what bench.py times: the production ring of ``FusedTwoTowerStep`` (T1 = EBC
gather + bf16-MFMA towers fwd/bwd-data + dot/BCE + in-place row-wise Adagrad of the rows looked up
once, from the dedup table the previous step built; tail = weight gradients + the next batch's
insert + row-wise Adagrad of the other rows; T3 = slab reduction + Adam) replayed from HIP graphs
over resident batches, with ``materialize_pooled`` so that T1 also writes the gathered rows and
every dX row for the checks; for config 5 the multi-hot KJT path (tt_pooled_fwd -> towers -> tiled
tt_bwd_prepare -> tt_bwd_rowwise_adagrad). Shapes:

  north star  100M items x 50M users, D 128, B 8192 (tables of 1.28e10 / 6.4e9 fp32 elements: far
              past 2^31, so every 64-bit row offset is exercised); uniform and Zipf ids
  config 2    10M items x 5M users, D 64, B 4096
  config 5    100M x 50M, D 128, B 16384, multi-hot bags of Uniform{1..39} ids (mean 20)

Two steps run; the second is checked, from a state the first one changed (non-zero Adagrad state,
Adam step 2). Each check feeds the oracle the kernels' OWN intermediate where the comparison would
otherwise be a bf16-tower comparison (the gradient rows dX that T1 writes):

* gathered rows (``materialize_pooled``): bit-exact against the table rows the transform selects
  (id 0 -> an empty bag, id % N, 03_model_training.py:356-365); multi-hot: the oracle's
  ``F.embedding_bag`` sum over the same rows, rtol 1e-6;
* towers: logits, dX and the tower gradients against the fp64 emulation of the kernels' rounding
  points (tests/tower_emul.py) ELEMENT-WISE: every element within its propagated error bound (the
  fp32 summation-order bound carried through the bf16 roundings, with ReLU units whose
  pre-activation lies within error of 0 marked ambiguous), plus per-row relative L2 error of dX
  <= 1e-2 and per-logit relative error <= 5e-3 on the rows without an ambiguous unit, gradient
  elements within 1e-3 of the tensor's max; loss rtol 1e-4. A negative case perturbs one dX row
  by 2 % and requires the checker to fail;
* the embedding update (T1's in-place rows + the tail's; tables + row-wise state of every touched
  row): ``oracle.rowwise_adagrad_from_lookups`` fed the EMULATED dX (not the kernels'), with a
  tolerance derived from the dX bounds (summed per row, through s += mean(G^2) and
  w -= lr G / (sqrt(s) + eps)) plus fp32 slack — eps 1e-10, lr 0.01 (03:791-795);
* Adam: the oracle's torch.optim.Adam restatement fed the kernels' own tower gradient, rtol 1e-5
  (absolute floors: 1e-6 x max|g| on the moments, 1e-5 x lr on the parameters, where m = 0.9 m0 +
  0.1 g cancels).
"""
import numpy as np
import pytest
import torch

from oracle import ref
from tower_emul import check_adagrad, check_towers, emulate_bounds, split_params

pytestmark = pytest.mark.gpu

LAYERS = [128, 64]
LR = 0.01
CASES = {
    "northstar": dict(N=[50_000_000, 100_000_000], D=128, B=8192),
    "config2": dict(N=[5_000_000, 10_000_000], D=64, B=4096),
}


def _zipf(g, n, N, device):
    u01 = torch.rand(n, generator=g, device=device, dtype=torch.float64)
    r = torch.floor(torch.exp(u01 * np.log(float(N))))
    return (r.to(torch.int64) * 2654435761) % N


def _single_hot_batches(N, B, ids, device, seed, n=2):
    g = torch.Generator(device=device).manual_seed(seed)
    out = []
    for _ in range(n):
        cols = []
        for n_ in N:
            if ids == "uniform":  # ids past N exercise the reference's id % N, zeros its drop
                c = torch.randint(0, 2 * n_, (B,), generator=g, device=device, dtype=torch.int64)
            else:
                c = _zipf(g, B, n_, device)
            c[torch.randint(0, B, (B // 64,), generator=g, device=device)] = 0
            cols.append(c)
        lab = torch.randint(0, 2, (B,), generator=g, device=device, dtype=torch.int32)
        out.append((cols, lab))
    return out


def _free():
    import gc

    gc.collect()
    torch.cuda.empty_cache()


def _grad_list(grads, prm):
    out, o = [], 0
    for p in prm:
        out.append(grads[o:o + p.numel()].reshape(p.shape))
        o += p.numel()
    return out


def _check_towers(xq, xc, params_before, st, labels, logits, gq, gc_, grads, B, negative=False):
    """Element-wise tower checks (tower_emul.check_towers); returns (params before, emulation)."""
    D_q, D_c = xq.shape[1], xc.shape[1]
    prm = split_params(params_before, [D_q, D_c], LAYERS)
    emu = emulate_bounds(xq, xc, prm, LAYERS, labels.cpu())
    stats = check_towers(emu, logits, [gq, gc_], _grad_list(grads, prm), "towers")
    print("tower check:", stats)
    np.testing.assert_allclose(float(st.loss), float(emu[1]), rtol=1e-4)
    if negative:  # the checker bites: one dX row (no ambiguous ReLU unit) 2 % off must fail it
        row = int((~emu[4]).nonzero()[len(logits) // 3])
        for t, g in enumerate((gq, gc_)):
            bad = [gq.clone(), gc_.clone()]
            bad[t][row] *= 1.02
            with pytest.raises(AssertionError):
                check_towers(emu, logits, bad, _grad_list(grads, prm), "negative")
    return prm, emu


def _check_adam(prm_before, grads, m0, v0, step0, params_after, exp_avg_after, exp_avg_sq_after):
    """torch.optim.Adam (03_model_training.py:826-829) fed the kernels' tower gradient."""
    shapes = [p.shape for p in prm_before]
    ps, gs, ms, vs, o = [], [], [], [], 0
    for s in shapes:
        n = int(np.prod(s))
        ps.append(torch.cat([p.reshape(-1) for p in prm_before])[o:o + n].clone())
        gs.append(grads[o:o + n].clone())
        ms.append(m0[o:o + n].clone())
        vs.append(v0[o:o + n].clone())
        o += n
    ref.adam(ps, gs, ms, vs, step0 + 1, LR)
    # the moments and the step may cancel (m = 0.9 m0 + 0.1 g): absolute floors relative to the
    # gradient scale and to the step size lr (an Adam step moves a parameter by at most ~lr)
    gmax = float(grads.abs().max())
    np.testing.assert_allclose(exp_avg_after.numpy(), torch.cat(ms).numpy(), rtol=1e-5, atol=1e-6 * gmax)
    np.testing.assert_allclose(exp_avg_sq_after.numpy(), torch.cat(vs).numpy(), rtol=1e-5, atol=1e-6 * gmax ** 2)
    np.testing.assert_allclose(params_after.numpy(), torch.cat(ps).numpy(), rtol=1e-5, atol=1e-5 * LR)


def _check_rowwise_adagrad(table_view, state_view, u, w_before, s_before, lookup_rows, dx_want, dx_bound):
    """The embedding update on the touched rows only (``u`` device, unique rows; ``lookup_rows``
    CPU, the row of every kept lookup in lookup order) against the oracle fed the EMULATED dX rows,
    tolerance from their bounds (tower_emul.check_adagrad)."""
    inv = torch.searchsorted(u.cpu(), lookup_rows)
    w_got = table_view[u].cpu()
    rel = check_adagrad(w_got, state_view[u].cpu(), w_before, s_before, inv, dx_want, dx_bound, LR, 1e-10, "adagrad")
    assert not torch.equal(w_got, w_before)  # the update happened
    print(f"adagrad check: median tolerance / step {rel:.3g}")


@pytest.mark.parametrize("case,ids", [("northstar", "uniform"), ("northstar", "zipf"), ("config2", "uniform")])
def test_production_step_at_baseline_size(device, case, ids):
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    N, D, B = CASES[case]["N"], CASES[case]["D"], CASES[case]["B"]
    st = FusedTwoTowerStep(N, [D, D], [0], [1], LAYERS, B, device, lr_emb=LR, lr_dense=LR, id_dtype=torch.int64,
                           seed=0, materialize_pooled=True)
    # the production configuration bench.py times: the ring (fused gather + single-hot dedup)
    assert st.towers is not None and st.ring_supported()
    if case == "northstar":
        assert st.tables.rows[1] * D > 2 ** 31 and st.tables.weight_offsets[1] > 2 ** 31
    batches = _single_hot_batches(N, B, ids, device, seed=11 if ids == "uniform" else 12)
    st.capture_ring(batches, steps_per_graph=1)
    st.run(1)
    torch.cuda.synchronize()
    cols, lab = batches[1]
    # state before step 2 (touched rows only; the tables themselves stay on the GPU)
    keep = [c != 0 for c in cols]
    rows = [c[k] % n for c, k, n in zip(cols, keep, N)]
    uniq = [torch.unique(r) for r in rows]
    before = [(st.tables.table_view(t)[uniq[t]].cpu(), st.tables.state_view(t)[uniq[t]].cpu()) for t in range(2)]
    params0, m0, v0 = st.params.cpu().clone(), st.exp_avg.cpu().clone(), st.exp_avg_sq.cpu().clone()
    step0 = int(st.adam_state[0])
    assert step0 == 1
    st.run(1)
    torch.cuda.synchronize()
    # (1) gathered rows: bit-exact (id 0 -> zeros)
    pooled = st.pooled.cpu()
    for t in range(2):
        want = torch.zeros(B, D)
        want[keep[t].cpu()] = before[t][0][torch.searchsorted(uniq[t].cpu(), rows[t].cpu())]
        assert torch.equal(pooled[:, t * D:(t + 1) * D], want), f"table {t}: gathered rows differ"
    # (2) towers vs the fp64 emulation of the kernels' rounding points
    gp = st.gpooled.cpu()
    grads = st.grads.cpu()
    prm, emu = _check_towers(pooled[:, :D], pooled[:, D:], params0, st, lab, st.logits.cpu(), gp[:, :D], gp[:, D:],
                             grads, B, negative=(case == "northstar" and ids == "uniform"))
    dxs = emu[2]
    # (3) row-wise Adagrad (T1 in place + tail) against the oracle fed the EMULATED dX rows (lookup
    # i = (feature, bag), kept lookups), tolerance from their bounds
    for t in range(2):
        k = keep[t].cpu()
        _check_rowwise_adagrad(st.tables.table_view(t), st.tables.state_view(t), uniq[t], before[t][0], before[t][1],
                               rows[t].cpu(), dxs[t][0][k].contiguous(), dxs[t][1][k].contiguous())
    # (4) Adam on the towers, fed the kernels' tower gradient
    _check_adam(prm, grads, m0, v0, step0, st.params.cpu(), st.exp_avg.cpu(), st.exp_avg_sq.cpu())
    del st, batches
    _free()


def _kjt_batches(N, B, maxlen, device, seed, n=2):
    g = torch.Generator(device=device).manual_seed(seed)
    out = []
    for _ in range(n):
        lengths = torch.randint(1, maxlen + 1, (2 * B,), generator=g, device=device, dtype=torch.int32)
        offsets = torch.zeros(2 * B + 1, dtype=torch.int32, device=device)
        offsets[1:] = torch.cumsum(lengths, 0)
        vals = [torch.randint(0, n_, (int(lengths[f * B:(f + 1) * B].sum()),), generator=g, device=device,
                              dtype=torch.int64) for f, n_ in enumerate(N)]
        lab = torch.randint(0, 2, (B,), generator=g, device=device, dtype=torch.int32)
        out.append((torch.cat(vals), offsets, lab))
    return out


def test_production_multihot_step_config5(device):
    """SURVEY §8(d) config 5 on one GPU: 100M x 50M, D 128, B 16384, bags U{1..39}."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    N, D, B = [50_000_000, 100_000_000], 128, 16384
    batches = _kjt_batches(N, B, 39, device, seed=4)
    cap = max(v.numel() for v, _, _ in batches)
    st = FusedTwoTowerStep(N, [D, D], [0], [1], LAYERS, B, device, lr_emb=LR, lr_dense=LR, id_dtype=torch.int64,
                           seed=0, max_lookups=cap, materialize_pooled=True)
    assert st.towers is not None and st.kjt_input and st.gather_kjt  # sum pool inside T1
    st.capture_pool_kjt(batches)
    st.pool_graphs[0].replay()
    torch.cuda.synchronize()
    vals, offs, lab = batches[1]
    o = offs.cpu().to(torch.int64)
    seg = [(int(o[f * B]), int(o[(f + 1) * B])) for f in range(2)]
    rows = [vals[s:e] for s, e in seg]
    uniq = [torch.unique(r) for r in rows]
    before = [(st.tables.table_view(t)[uniq[t]].cpu(), st.tables.state_view(t)[uniq[t]].cpu()) for t in range(2)]
    params0, m0, v0 = st.params.cpu().clone(), st.exp_avg.cpu().clone(), st.exp_avg_sq.cpu().clone()
    step0 = int(st.adam_state[0])
    st.pool_graphs[1].replay()
    torch.cuda.synchronize()
    pooled, gp, grads = st.pooled.cpu(), st.gpooled.cpu(), st.grads.cpu()
    inv = [torch.searchsorted(uniq[t].cpu(), rows[t].cpu()) for t in range(2)]
    for t in range(2):
        bag_off = (o[t * B:(t + 1) * B + 1] - o[t * B])
        want = torch.nn.functional.embedding_bag(inv[t], before[t][0], bag_off, mode="sum", include_last_offset=True)
        np.testing.assert_allclose(pooled[:, t * D:(t + 1) * D].numpy(), want.numpy(), rtol=1e-6, atol=1e-7)
    prm, emu = _check_towers(pooled[:, :D], pooled[:, D:], params0, st, lab, st.logits.cpu(), gp[:, :D], gp[:, D:],
                             grads, B)
    dxs = emu[2]
    for t in range(2):
        lens = o[t * B + 1:(t + 1) * B + 1] - o[t * B:(t + 1) * B]
        bag = torch.repeat_interleave(torch.arange(B), lens)
        _check_rowwise_adagrad(st.tables.table_view(t), st.tables.state_view(t), uniq[t], before[t][0], before[t][1],
                               rows[t].cpu(), dxs[t][0][bag].contiguous(), dxs[t][1][bag].contiguous())
    _check_adam(prm, grads, m0, v0, step0, st.params.cpu(), st.exp_avg.cpu(), st.exp_avg_sq.cpu())
    del st, batches
    _free()
