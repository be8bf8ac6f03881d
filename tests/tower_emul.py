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


def rel_err(got: torch.Tensor, want: torch.Tensor) -> float:
    got, want = got.double().reshape(-1), want.double().reshape(-1)
    return float((got - want).norm() / (want.norm() + 1e-30))
