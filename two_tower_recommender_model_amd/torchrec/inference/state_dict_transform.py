"""torchrec.inference.state_dict_transform (imported at 03_model_training.py:335-338)."""
from __future__ import annotations

from typing import Dict

import torch


def state_dict_gather(src: Dict[str, torch.Tensor], dst: Dict[str, torch.Tensor]) -> None:
    """Copy every tensor of ``src`` into ``dst`` (local tensors; gathers ShardedTensors to dst)."""
    for k, v in src.items():
        if hasattr(v, "gather") and not isinstance(v, torch.Tensor):
            v.gather(0, dst[k])
        else:
            dst[k].copy_(v)


def state_dict_to_device(state_dict: Dict[str, torch.Tensor], pg=None, device=None) -> Dict[str, torch.Tensor]:
    return {k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in state_dict.items()}
