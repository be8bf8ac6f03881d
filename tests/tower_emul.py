"""fp64 emulation of the fused bf16 tower kernels' rounding points (test infrastructure).

The towers are torchrec MLPs (Linear + ReLU on every layer, 03_model_training.py:411-412) over the
tower inputs, then logits = (q * c).sum(1) and BCEWithLogits(mean) (03:452-453). The kernels round
the layer inputs X, the weights W, the hidden activations and every dZ to bf16 and accumulate in
fp32; the last layer's outputs stay fp32, bias gradients sum the unrounded dZ. This module replays
exactly those rounding points in fp64, so a kernel is checked on its arithmetic, not on ReLU masks
that flip where a pre-activation is within bf16 error of 0 (which a plain fp32 autograd comparison
would be dominated by).
"""
from __future__ import annotations

from typing import List, Sequence

import torch


def bf(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.bfloat16).double()


def split_params(flat: torch.Tensor, in_dims: Sequence[int], widths: Sequence[int]) -> List[torch.Tensor]:
    """Flat parameter buffer -> [qW0, qb0, qW1, qb1, ..., cW0, cb0, ...] (tt_tower_shape_t layout)."""
    out, o = [], 0
    flat = flat.detach().cpu()
    for t in range(2):
        k = in_dims[t]
        for w in widths:
            out.append(flat[o:o + w * k].view(w, k).clone())
            o += w * k
            out.append(flat[o:o + w].clone())
            o += w
            k = w
    assert o == flat.numel(), (o, flat.numel())
    return out


def emulate(xq: torch.Tensor, xc: torch.Tensor, params: Sequence[torch.Tensor], widths: Sequence[int],
            labels: torch.Tensor):
    """Returns (logits [B], loss, [dXq, dXc], grads in params order), all fp64."""
    B = xq.shape[0]
    L = len(widths)
    Ws = [bf(p) if p.dim() == 2 else p.double() for p in params]
    acts, outs = [], []
    i = 0
    for x in (xq, xc):
        h = bf(x)
        a_t = [h]
        for li in range(L):
            z = torch.relu(h @ Ws[i].T + Ws[i + 1])
            i += 2
            h = z if li == L - 1 else bf(z)
            a_t.append(h)
        acts.append(a_t)
        outs.append(h.float().double())
    logits = (outs[0] * outs[1]).sum(1)
    y = labels.double()
    loss = torch.nn.functional.binary_cross_entropy_with_logits(logits, y)
    dl = (torch.sigmoid(logits) - y) / B
    grads, dxs = [], []
    for t in range(2):
        dz = dl[:, None] * outs[1 - t] * (outs[t] > 0)
        g_t = [None] * (2 * L)
        for li in reversed(range(L)):
            Wi = Ws[t * 2 * L + 2 * li]
            g_t[2 * li] = bf(dz).T @ acts[t][li]
            g_t[2 * li + 1] = dz.sum(0)
            dA = bf(dz) @ Wi
            dz = dA * (acts[t][li] > 0) if li > 0 else dA
        dxs.append(dz)
        grads += g_t
    return logits, loss, dxs, grads


U32 = 2.0 ** -24  # fp32 unit roundoff


LAMBDA = 8.0


def acc_err(terms_l2: torch.Tensor, total: torch.Tensor, n: int) -> torch.Tensor:
    """Bound on the rounding error of an fp32 sum of n terms, in any order: LAMBDA x u x sqrt(n) x
    (||terms||_2 + |sum|). Each partial sum S_k carries a rounding error of at most u |S_k|; for
    terms of either sign the partial sums grow like a random walk plus the drift toward the total
    (|S_k| <~ sqrt(k) rms + (k / n) |sum|), and the rounding errors of the n additions do not all
    share one sign, so their sum stays within a few u sqrt(sum_k S_k^2) <= u sqrt(n) (||terms||_2 +
    |sum|) (the probabilistic view of Higham & Mary, SIAM J. Sci. Comput. 41(5), 2019). LAMBDA = 8
    keeps ~20 standard deviations of margin; the worst case n u sum|terms| assumes every error has
    the same sign, is ~sqrt(n) times looser and would swamp the check."""
    return LAMBDA * U32 * n ** 0.5 * (terms_l2 + total.abs())


def _mm_err(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, n: int) -> torch.Tensor:
    """acc_err of out = a @ b (n terms per element)."""
    return acc_err(((a * a) @ (b * b)).sqrt(), out, n)


def _bf32(x: torch.Tensor) -> torch.Tensor:
    """bf16 rounding of an fp32 value (what the kernels do to their fp32 accumulators)."""
    return x.float().to(torch.bfloat16).double()


def _round_err(v: torch.Tensor, e: torch.Tensor, fn=_bf32) -> torch.Tensor:
    """Bound on |fn(v') - fn(v)| for every v' in [v - e, v + e], fn monotone (bf16 rounding, with or
    without a ReLU in front): exact, since fn(v') lies in [fn(v - e), fn(v + e)]. Zero where the
    whole interval rounds to one value."""
    c = fn(v)
    return torch.maximum((fn(v + e) - c).abs(), (fn(v - e) - c).abs())


def _relu_bf(v):
    return _bf32(torch.relu(v))


def emulate_bounds(xq: torch.Tensor, xc: torch.Tensor, params: Sequence[torch.Tensor], widths: Sequence[int],
                   labels: torch.Tensor, ex=None):
    """``emulate`` plus a per-element bound on how far the kernels' values may lie from it.

    The kernels and the emulation share every rounding point; they differ only in the order of the
    fp32 sums. Each sum of n terms is off by at most gamma(n) x (sum of |terms|) (any order), and
    the bound is carried through every later operation: through products (|a| e_b + e_a |b| +
    e_a e_b), through the bf16 roundings (an exact interval: a rounding moves only where the
    interval straddles a rounding boundary — otherwise both round to the same bf16), and through
    the ReLU masks (where a pre-activation's interval contains 0 the mask is ambiguous and the
    bound takes the whole value: the explicit mask for ReLU flips within error of 0). The last
    layer's sigmoid uses the hardware exp / reciprocal: 1e-6 absolute on sigma is allowed.

    ``ex`` (optional) = [e_xq, e_xc]: element-wise bounds on how far the kernels' tower inputs may
    lie from xq / xc (multi-hot bags: the pooled sums are fp32 sums in another order); by default
    the inputs are the same values (single-hot rows).

    Returns (logits, e_logits), loss, [(dX, e_dX) per tower], [(g, e_g) in params order], all
    fp64, and ``ambiguous`` [B] bool: the rows with a ReLU unit (either tower, any layer) whose
    pre-activation lies within its bound of 0 (their mask may differ from the kernels').
    """
    B = xq.shape[0]
    L = len(widths)
    Ws = [bf(p) if p.dim() == 2 else p.double() for p in params]
    acts, zs, ezs, eacts, outs, eouts = [], [], [], [], [], []
    ambiguous = torch.zeros(B, dtype=torch.bool)
    i = 0
    for t_in, x in enumerate((xq, xc)):
        if ex is None:
            h = bf(x)
            eh = torch.zeros_like(h)
        else:
            x = x.double()
            h = _bf32(x)
            eh = _round_err(x, ex[t_in].double())
        a_t, ea_t, z_t, ez_t = [h], [eh], [], []
        for li in range(L):
            W, b = Ws[i], Ws[i + 1]
            i += 2
            K = W.shape[1]
            z = h @ W.T + b
            ha = h.abs() + eh
            ez = eh @ W.abs().T + acc_err(((ha * ha) @ (W * W).T + b * b).sqrt(), z, K + 1)
            z_t.append(z)
            ez_t.append(ez)
            if li == L - 1:
                ambiguous |= (z.abs() <= ez).any(1)
            else:
                ambiguous |= ((_relu_bf(z - ez) == 0) & (_relu_bf(z + ez) > 0)).any(1)
            if li == L - 1:  # fp32 outputs
                h, eh = torch.relu(z), ez + U32 * z.abs()
            else:
                h, eh = _relu_bf(z), _round_err(z, ez, _relu_bf)
            a_t.append(h)
            ea_t.append(eh)
        acts.append(a_t)
        eacts.append(ea_t)
        zs.append(z_t)
        ezs.append(ez_t)
        outs.append(h.float().double())
        eouts.append(eh)
    q, c = outs
    eq, ec = eouts
    logits = (q * c).sum(1)
    e_log = (eq * c.abs() + q.abs() * ec + eq * ec).sum(1) + \
        acc_err((((q.abs() + eq) * (c.abs() + ec)) ** 2).sum(1).sqrt(), logits, q.shape[1])
    y = labels.double()
    loss = torch.nn.functional.binary_cross_entropy_with_logits(logits, y)
    dl = (torch.sigmoid(logits) - y) / B
    e_dl = (0.25 * e_log + 1e-6) / B
    grads, dxs = [], []
    for t in range(2):
        oo, eoo = outs[1 - t], eouts[1 - t]
        zl, ezl = zs[t][L - 1], ezs[t][L - 1]
        prod = dl[:, None] * oo
        e_prod = e_dl[:, None] * oo.abs() + dl.abs()[:, None] * eoo + e_dl[:, None] * eoo + 2 * U32 * prod.abs()
        on = zl > 0
        ambig = zl.abs() <= ezl
        dz = prod * on
        edz = torch.where(ambig, prod.abs() + e_prod, torch.where(on, e_prod, torch.zeros_like(e_prod)))
        g_t = [None] * (2 * L)
        for li in reversed(range(L)):
            Wi = Ws[t * 2 * L + 2 * li]
            a, ea = acts[t][li], eacts[t][li]
            bdz, ebdz = _bf32(dz), _round_err(dz, edz)
            gW = bdz.T @ a
            egW = ebdz.T @ a.abs() + bdz.abs().T @ ea + ebdz.T @ ea + \
                _mm_err((bdz.abs() + ebdz).T, a.abs() + ea, gW, B)
            gb = dz.sum(0)
            egb = edz.sum(0) + acc_err(((dz.abs() + edz) ** 2).sum(0).sqrt(), gb, B)
            g_t[2 * li], g_t[2 * li + 1] = (gW, egW), (gb, egb)
            K = Wi.shape[0]
            dA = bdz @ Wi
            edA = ebdz @ Wi.abs() + _mm_err(bdz.abs() + ebdz, Wi.abs(), dA, K)
            if li > 0:
                zp, ezp = zs[t][li - 1], ezs[t][li - 1]
                on = a > 0
                # the kernel's mask is its own bf16 activation > 0: ambiguous where the interval of
                # the activation holds both 0 and a positive value
                ambig = (_relu_bf(zp - ezp) == 0) & (_relu_bf(zp + ezp) > 0)
                dz = dA * on
                edz = torch.where(ambig, dA.abs() + edA, torch.where(on, edA, torch.zeros_like(edA)))
            else:
                dz, edz = dA, edA
        dxs.append((dz, edz))
        grads += g_t
    return (logits, e_log), loss, dxs, grads, ambiguous


def check_within(got: torch.Tensor, want: torch.Tensor, bound: torch.Tensor, what: str = "") -> None:
    """Element-wise |got - want| <= bound (+ the fp32 rounding of the stored value); raises an
    AssertionError naming the worst element and how many elements break the bound."""
    got, want, bound = got.double().reshape(-1), want.double().reshape(-1), bound.double().reshape(-1)
    lim = bound + 2 * U32 * want.abs() + 1e-30
    diff = (got - want).abs()
    bad = ~(diff <= lim)
    if bool(bad.any()):
        j = int(torch.argmax(torch.where(bad, diff / lim, torch.zeros_like(diff))))
        raise AssertionError(f"{what}: {int(bad.sum())} of {got.numel()} elements outside the bound; worst at "
                             f"{j}: got {float(got[j]):.9g}, want {float(want[j]):.9g}, |diff| {float(diff[j]):.3g} "
                             f"> bound {float(lim[j]):.3g}")


ROW_RTOL = 1e-2     # dX rows: relative L2 error (rows without an ambiguous ReLU unit)
LOGIT_RTOL = 5e-3   # logits: relative error (same rows)
GRAD_RTOL = 1e-3    # weight / bias gradients: error relative to the tensor's largest element


def check_towers(emu, logits, dx, grads, what: str = "") -> dict:
    """The towers' parity check (logits [B], dx = [dXq, dXc] each [B, in], grads in params order,
    each of its parameter's shape) against ``emulate_bounds`` output ``emu``, in two layers:

    (1) every element within its propagated bound (``check_within``): no false failures by
        construction, loose where a dZ element's bf16 rounding may go either way (a few % of dX);
    (2) tight per-row / per-element statistics on the rows without an ambiguous ReLU unit: each dX
        row's relative L2 error <= ROW_RTOL, each logit's relative error <= LOGIT_RTOL, each gradient
        element's error <= GRAD_RTOL x the tensor's largest |element|. Rounding flips between fp32
        summation orders stay ~10x below these (measured: dX rows <= 4e-3, logits <= 5.5e-4,
        gradients <= 3.8e-4 of max), so a localised error of ~1-2 % on one row is caught.
    Returns the worst ratios seen (for logs)."""
    (lg, e_lg), _, dxs, gw, amb = emu
    ok = ~amb
    check_within(logits, lg, e_lg, f"{what} logits")
    for t in range(2):
        check_within(dx[t], dxs[t][0], dxs[t][1], f"{what} dX[{t}]")
    for j, (want, e) in enumerate(gw):
        check_within(grads[j], want, e, f"{what} grad[{j}]")
    out = {"ambiguous_rows": int(amb.sum())}
    got_l, want_l = logits.double().reshape(-1)[ok], lg[ok]
    r = ((got_l - want_l).abs() / want_l.abs().clamp_min(1e-30))
    out["logit_rel_max"] = float(r.max()) if r.numel() else 0.0
    assert out["logit_rel_max"] <= LOGIT_RTOL, (what, "logits", out)
    for t in range(2):
        g, w = dx[t].double()[ok], dxs[t][0][ok]
        rr = (g - w).norm(dim=1) / w.norm(dim=1).clamp_min(1e-30)
        zero = w.norm(dim=1) == 0
        rr = torch.where(zero, (g - w).norm(dim=1), rr)
        out[f"dx{t}_row_rel_max"] = float(rr.max()) if rr.numel() else 0.0
        if out[f"dx{t}_row_rel_max"] > ROW_RTOL:
            j = int(rr.argmax())
            raise AssertionError(f"{what} dX[{t}]: row {int(ok.nonzero()[j])} relative error {float(rr[j]):.3g} > "
                                 f"{ROW_RTOL}")
    for j, (want, _) in enumerate(gw):
        m = float(want.abs().max())
        d = float((grads[j].double() - want).abs().max())
        out[f"grad{j}_rel_max"] = d / m if m else d
        assert d <= GRAD_RTOL * m + 1e-30, (what, f"grad[{j}]", out)
    return out


def check_adagrad(w_got, s_got, w_before, s_before, inv, dx_want, dx_bound, lr: float, eps: float = 1e-10,
                  what: str = "") -> float:
    """The row-wise Adagrad update (03_model_training.py:791-795) of U touched rows against the
    oracle (oracle.ref.rowwise_adagrad_from_lookups) fed the EMULATED gradient rows: lookup j adds
    dx_want[j] (element-wise bound dx_bound[j]) to touched row inv[j]. The tolerance is that bound
    carried through the update: G = sum of a row's lookups (e_G = sum of their bounds),
    s' = s + mean(G^2) (e_s = mean(2 |G| e_G + e_G^2)), w' = w - lr G / (sqrt(s') + eps)
    (e_w = lr (e_G / r_lo + |G| (1 / r_lo - 1 / r)), r_lo from s' - e_s), plus the update's own fp32
    arithmetic (1e-5 relative). w_* [U, D] and s_* [U] are CPU tensors. Returns the median
    tolerance relative to the step (for logs)."""
    from oracle import ref

    w_want, s_want = w_before.clone(), s_before.clone()
    ref.rowwise_adagrad_from_lookups(w_want, s_want, inv, dx_want.float(), lr, eps)
    n = w_before.shape[0]
    G = torch.zeros(n, dx_want.shape[1], dtype=torch.float64).index_add_(0, inv, dx_want.double())
    eG = torch.zeros_like(G).index_add_(0, inv, dx_bound.double())
    s_new = s_before.double() + (G * G).mean(1)
    e_s = (2 * G.abs() * eG + eG * eG).mean(1)
    r = s_new.sqrt() + eps
    r_lo = (s_new - e_s).clamp_min(0).sqrt() + eps
    e_w = lr * (eG / r_lo[:, None] + G.abs() * (1 / r_lo - 1 / r)[:, None])
    tol_s = e_s + 1e-5 * s_new.abs() + 1e-12
    bad = ~((s_got.double() - s_want.double()).abs() <= tol_s)
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} row-wise Adagrad states outside the bound"
    tol_w = e_w + 1e-5 * w_want.double().abs() + 1e-5 * lr * (G.abs() / r[:, None])
    bad = ~((w_got.double() - w_want.double()).abs() <= tol_w)
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} table elements outside the bound"
    return float((e_w / (lr * G.abs() / r[:, None]).clamp_min(1e-30)).median())


def check_adam(p_before, m_before, v_before, step: int, g, e_g, p_got, m_got, v_got, lr: float,
               betas=(0.9, 0.999), eps: float = 1e-8, what: str = "") -> None:
    """torch.optim.Adam (KeyedOptimizerWrapper(Adam), 03_model_training.py:826-829) on flat fp32
    parameters: step ``step`` (1-based) from (p, m, v)_before with the EMULATED gradient g, bound
    e_g, against the kernels' (p, m, v) after. The bound is carried through m' = b1 m + (1 - b1) g,
    v' = b2 v + (1 - b2) g^2 and the update lr m^ / (sqrt(v^) + eps), plus fp32 slack."""
    b1, b2 = betas
    g, e_g = g.double(), e_g.double()
    m = b1 * m_before.double() + (1 - b1) * g
    v = b2 * v_before.double() + (1 - b2) * g * g
    e_m = (1 - b1) * e_g
    e_v = (1 - b2) * (2 * g.abs() * e_g + e_g * e_g)
    c1, c2 = 1 - b1 ** step, 1 - b2 ** step
    mh, vh, e_mh, e_vh = m / c1, v / c2, e_m / c1, e_v / c2
    den = vh.sqrt() + eps
    den_lo = (vh - e_vh).clamp_min(0).sqrt() + eps
    p = p_before.double() - lr * mh / den
    e_p = lr * (e_mh / den_lo + mh.abs() * (1 / den_lo - 1 / den))
    for name, got, want, e in (("exp_avg", m_got, m, e_m), ("exp_avg_sq", v_got, v, e_v), ("param", p_got, p, e_p)):
        lim = e + 1e-5 * want.abs() + (1e-6 * lr if name == "param" else 1e-30)
        bad = ~((got.double() - want).abs() <= lim)
        if bool(bad.any()):
            idx = torch.nonzero(bad).flatten()[:6].tolist()
            detail = "; ".join(f"[{i}] got {float(got[i]):.9g} want {float(want[i]):.9g} lim {float(lim[i]):.3g} "
                               f"g {float(g[i]):.4g} e_g {float(e_g[i]):.3g}" for i in idx)
            raise AssertionError(f"{what} Adam {name}: {int(bad.sum())} of {want.numel()} outside the bound: {detail}")


def rel_err(got: torch.Tensor, want: torch.Tensor) -> float:
    got, want = got.double().reshape(-1), want.double().reshape(-1)
    return float((got - want).norm() / (want.norm() + 1e-30))
