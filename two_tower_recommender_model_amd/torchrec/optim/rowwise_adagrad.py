"""torchrec.optim.rowwise_adagrad.RowWiseAdagrad — the optimizer class the reference attaches to
the EBC tables with ``_apply_optimizer_in_backward`` (03_model_training.py:791-795).

On the MI355X path this class is a DESCRIPTOR: EmbeddingBagCollection reads its hyper-parameters
from the tables' ``_optimizer_classes/_optimizer_kwargs`` and applies the update inside the fused
backward kernel (the Parameters never receive a ``.grad``, so ``step()`` below is not reached).
``step()`` is the plain algorithm for any parameter that does get a dense gradient:
  state[r] += mean_d g[r,d]^2 ; w[r] += (-lr * g[r]) / (sqrt(state[r]) + eps)
(lr default 1e-2, eps 1e-10, lr_decay / weight_decay 0, initial accumulator 0).
"""
from __future__ import annotations

from typing import Any, Dict, Iterable

import torch
from torch.optim.optimizer import Optimizer


class RowWiseAdagrad(Optimizer):
    def __init__(self, params: Iterable[torch.Tensor], lr: float = 1e-2, lr_decay: float = 0.0,
                 weight_decay: float = 0.0, initial_accumulator_value: float = 0.0, eps: float = 1e-10,
                 *, maximize: bool = False, **unused: Any) -> None:
        if lr < 0 or eps < 0 or lr_decay < 0 or weight_decay < 0 or initial_accumulator_value < 0:
            raise ValueError("invalid RowWiseAdagrad hyper-parameter")
        defaults = dict(lr=lr, lr_decay=lr_decay, eps=eps, weight_decay=weight_decay,
                        initial_accumulator_value=initial_accumulator_value, maximize=maximize)
        super().__init__(params, defaults)
        for group in self.param_groups:
            for p in group["params"]:
                st = self.state[p]
                st["step"] = torch.tensor(0.0)
                st["sum"] = torch.full((p.shape[0], 1), initial_accumulator_value, dtype=p.dtype, device=p.device)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad if not group["maximize"] else -p.grad
                st = self.state[p]
                st["step"] += 1
                step = float(st["step"])
                row = g.pow(2).mean(dim=1, keepdim=True)
                if group["weight_decay"] != 0:
                    g = g.add(p, alpha=group["weight_decay"])
                clr = group["lr"] / (1 + (step - 1) * group["lr_decay"])
                st["sum"].add_(row)
                std = st["sum"].sqrt().add_(group["eps"])
                p.addcdiv_(g, std, value=-clr)
        return loss
