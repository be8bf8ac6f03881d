"""torchrec.distributed.comm subset (``get_local_size`` is called at 03_model_training.py:800)."""
from __future__ import annotations

import os
from typing import Optional

import torch.distributed as dist


def get_local_size(world_size: Optional[int] = None) -> int:
    if world_size is None:
        world_size = dist.get_world_size() if dist.is_initialized() else 1
    return int(os.environ.get("LOCAL_WORLD_SIZE", world_size))


def get_local_rank(world_size: Optional[int] = None, rank: Optional[int] = None) -> int:
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"])
    if rank is None:
        rank = dist.get_rank() if dist.is_initialized() else 0
    return rank % get_local_size(world_size)


def get_group_rank(world_size: Optional[int] = None, rank: Optional[int] = None) -> int:
    if rank is None:
        rank = dist.get_rank() if dist.is_initialized() else 0
    return rank // get_local_size(world_size)


def get_num_groups(world_size: Optional[int] = None) -> int:
    if world_size is None:
        world_size = dist.get_world_size() if dist.is_initialized() else 1
    return world_size // get_local_size(world_size)
