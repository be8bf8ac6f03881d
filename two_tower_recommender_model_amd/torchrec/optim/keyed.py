"""torchrec.optim.keyed.KeyedOptimizerWrapper — ``KeyedOptimizerWrapper(dict(model.named_parameters()),
lambda params: torch.optim.Adam(params, lr))`` (03_model_training.py:826-829). Tables whose update
is fused into the backward have ``grad is None`` and are skipped by the wrapped optimizer, so in the
reference setup it updates the MLP towers only."""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Mapping

import torch
from torch.optim.optimizer import Optimizer


class KeyedOptimizer(Optimizer):
    def __init__(self, params: Mapping[str, torch.Tensor], state: Mapping[Any, Any], param_groups):
        torch._C._log_api_usage_once(f"torchrec.optim.{self.__class__.__name__}")
        self.state = state
        self.param_groups = param_groups
        self.params = params
        self.defaults = {"_save_param_groups": False}

    def step(self, closure=None):  # pragma: no cover - overridden
        raise NotImplementedError


class KeyedOptimizerWrapper(KeyedOptimizer):
    def __init__(self, params: Mapping[str, torch.Tensor],
                 optim_factory: Callable[[List[torch.Tensor]], Optimizer]) -> None:
        self._optimizer = optim_factory(list(params.values()))
        super().__init__(params, self._optimizer.state, self._optimizer.param_groups)

    def zero_grad(self, set_to_none: bool = True) -> None:
        self._optimizer.zero_grad(set_to_none=set_to_none)

    def step(self, closure: Any = None) -> Any:
        return self._optimizer.step(closure=closure)

    def state_dict(self) -> Dict[str, Any]:
        return self._optimizer.state_dict()

    def load_state_dict(self, state_dict) -> None:
        self._optimizer.load_state_dict(state_dict)
