"""The per-element error bounds of tests/tower_emul.py (the towers' parity checker), on CPU.

(1) A stand-in for the kernels — the same rounding points evaluated in fp32 arithmetic, whose sums
    run in another order than the fp64 emulation's — lies inside the bounds on every element of
    the logits, dX and the weight / bias gradients (the bounds are not too tight).
(2) The checker bites: one row of dX off by 1 %, one logit off by 1e-3 relative or one weight-
    gradient element off by 1 % is reported (the bounds are not too loose: the round-2 relative
    Frobenius check let a 10 % error on one of 8192 rows through)."""
import pytest
import torch

from tower_emul import check_towers, check_within, emulate_bounds, split_params


def _fp32_towers(xq, xc, params, widths, labels):
    """The towers with the kernels' rounding points (bf16 X, W, hidden activations and dZ; fp32
    accumulation; fp32 last-layer outputs; bias gradients from the unrounded dZ), in fp32."""
    bf = lambda t: t.float().to(torch.bfloat16).float()  # noqa: E731
    B, L = xq.shape[0], len(widths)
    Ws = [bf(p) if p.dim() == 2 else p.float() for p in params]
    acts, outs, i = [], [], 0
    for x in (xq, xc):
        h = bf(x)
        a_t = [h]
        for li in range(L):
            z = torch.relu(h @ Ws[i].T + Ws[i + 1])
            i += 2
            h = z if li == L - 1 else bf(z)
            a_t.append(h)
        acts.append(a_t)
        outs.append(h)
    logits = (outs[0] * outs[1]).sum(1)
    dl = (torch.sigmoid(logits) - labels.float()) / B
    grads, dxs = [], []
    for t in range(2):
        dz = dl[:, None] * outs[1 - t] * (outs[t] > 0)
        g_t = [None] * (2 * L)
        for li in reversed(range(L)):
            g_t[2 * li] = bf(dz).T @ acts[t][li]
            g_t[2 * li + 1] = dz.sum(0)
            dA = bf(dz) @ Ws[t * 2 * L + 2 * li]
            dz = dA * (acts[t][li] > 0) if li > 0 else dA
        dxs.append(dz)
        grads += g_t
    return logits, dxs, grads


def _case(B, D, widths, seed):
    g = torch.Generator().manual_seed(seed)
    xq = torch.empty(B, D).uniform_(-0.3, 0.3, generator=g)
    xc = torch.empty(B, D).uniform_(-0.3, 0.3, generator=g)
    flat = []
    for _ in range(2):
        k = D
        for w in widths:
            flat += [torch.empty(w * k).uniform_(-k ** -0.5, k ** -0.5, generator=g),
                     torch.empty(w).uniform_(-k ** -0.5, k ** -0.5, generator=g)]
            k = w
    params = split_params(torch.cat(flat), [D, D], widths)
    labels = torch.randint(0, 2, (B,), generator=g)
    return xq, xc, params, labels


@pytest.mark.parametrize("B,D,widths,seed", [(2048, 128, [128, 64], 0), (1024, 64, [128, 64], 1),
                                             (512, 1024, [128, 64], 2)])
def test_fp32_stand_in_within_bounds(B, D, widths, seed):
    xq, xc, params, labels = _case(B, D, widths, seed)
    emu = emulate_bounds(xq, xc, params, widths, labels)
    (lg, e_lg), _, dxs, gw, amb = emu
    got_lg, got_dx, got_g = _fp32_towers(xq, xc, params, widths, labels)
    stats = check_towers(emu, got_lg, got_dx, got_g, "fp32 stand-in")
    assert stats["ambiguous_rows"] < B // 10
    # not vacuous: the median bound on dX is a few percent of the value (it is set by the dZ
    # elements whose bf16 rounding may go either way), and the stand-in's worst element uses a
    # sizeable share of its bound (the bound is not padded by orders of magnitude)
    for t in range(2):
        rel = (dxs[t][1] / dxs[t][0].abs().clamp_min(1e-30)).flatten().median()
        assert float(rel) < (0.1 if D <= 128 else 0.5)


@pytest.mark.parametrize("D", [128, 1024])
def test_checker_catches_one_bad_element(D):
    B = 2048 if D == 128 else 512
    xq, xc, params, labels = _case(B, D, [128, 64], 3)
    emu = emulate_bounds(xq, xc, params, [128, 64], labels)
    amb = emu[4]
    got_lg, got_dx, got_g = _fp32_towers(xq, xc, params, [128, 64], labels)
    check_towers(emu, got_lg, got_dx, got_g)
    row = int((~amb).nonzero()[B // 3])
    for t in range(2):  # one dX row 2 % off
        bad = [x.clone() for x in got_dx]
        bad[t][row] *= 1.02
        with pytest.raises(AssertionError, match="dX"):
            check_towers(emu, got_lg, bad, got_g)
    bad = got_lg.clone()  # one logit 1 % off
    bad[row] *= 1.01
    with pytest.raises(AssertionError):
        check_towers(emu, bad, got_dx, got_g)
    for j in (0, 4):  # one weight-gradient element 1 % of the tensor's largest off
        bad = [g.clone() for g in got_g]
        bad[j].view(-1)[17] += 0.01 * float(bad[j].abs().max())
        with pytest.raises(AssertionError):
            check_towers(emu, got_lg, got_dx, bad)
