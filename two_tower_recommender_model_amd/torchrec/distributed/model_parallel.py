"""torchrec.distributed.model_parallel.DistributedModelParallel on MI355X.

``DistributedModelParallel(module=train_task, device=device)`` (03_model_training.py:812-815):
one process per GPU. The module's EmbeddingBagCollections are placed by the sharding plan (the
reference builds no plan argument, so the default planner runs, 03:809-815): with a process group
(the reference always initialises one, 03:751) each is replaced by a ShardedEmbeddingBagCollection
(table-wise / row-wise shards, RCCL all-to-all and reduce-scatter over xGMI) — at world size 1 too,
as torchrec does; without one (single-process use) the tables are materialised on the device (meta
tables get torchrec's default init). Dense modules are replicated: parameters broadcast from rank 0 and
gradients all-reduced (averaged) by torch DDP with the table parameters excluded, as torchrec does.
"""
from __future__ import annotations

from typing import Any, Dict, Iterator, List, Optional, Tuple

import torch
import torch.distributed as dist
from torch import nn

from ..modules.embedding_modules import EmbeddingBagCollection
from .embeddingbag import EmbeddingBagCollectionSharder, ShardedEmbeddingBagCollection
from .planner import EmbeddingShardingPlanner, Topology
from .types import ShardingPlan


def get_default_sharders() -> List[Any]:
    return [EmbeddingBagCollectionSharder()]


def _set_submodule(root: nn.Module, path: str, new: nn.Module) -> None:
    parent = root
    parts = path.split(".")
    for p in parts[:-1]:
        parent = getattr(parent, p)
    setattr(parent, parts[-1], new)


class DistributedModelParallel(nn.Module):
    def __init__(self, module: nn.Module, env=None, device: Optional[torch.device] = None,
                 plan: Optional[ShardingPlan] = None, sharders: Optional[List[Any]] = None,
                 init_data_parallel: bool = True, init_parameters: bool = True, data_parallel_wrapper=None):
        super().__init__()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self._pg = dist.group.WORLD if dist.is_initialized() else None
        self._world_size = dist.get_world_size() if dist.is_initialized() else 1
        self._rank = dist.get_rank() if dist.is_initialized() else 0
        self._sharders = sharders or get_default_sharders()
        if plan is None:
            planner = EmbeddingShardingPlanner(topology=Topology(world_size=self._world_size,
                                                                 compute_device=self.device.type))
            plan = planner.collective_plan(module, self._sharders, self._pg)
        self._plan = plan
        self._sharded_paths: List[str] = []
        for path, ebc in [(n, m) for n, m in module.named_modules() if isinstance(m, EmbeddingBagCollection)]:
            mplan = plan.get_plan_for_module(path) or {}
            if self._pg is None:
                ebc._materialize(self.device)
            else:
                backend = next((getattr(sh, "lookup_backend", None) for sh in self._sharders
                                if getattr(sh, "lookup_backend", None) is not None), None)
                sharded = ShardedEmbeddingBagCollection(ebc, mplan, self._pg, self.device, backend=backend)
                if path == "":
                    module = sharded
                else:
                    _set_submodule(module, path, sharded)
                self._sharded_paths.append(path)
        # dense parameters -> device (embedding storage is already there)
        for name, p in module.named_parameters():
            if p.device != self.device and not _is_table_param(module, name):
                p.data = p.data.to(self.device)
        for name, b in module.named_buffers():
            if b.device != self.device:
                b.data = b.data.to(self.device)
        self._dmp_wrapped_module = module
        self._ddp = None
        if self._world_size > 1 and init_data_parallel:
            ignore = [n for n, _ in module.named_parameters() if _is_table_param(module, n)]
            ignore += [n for n, _ in module.named_buffers() if _is_table_param(module, n)]
            nn.parallel.DistributedDataParallel._set_params_and_buffers_to_ignore_for_model(module, ignore)
            dense = [p for n, p in module.named_parameters() if n not in ignore and p.requires_grad]
            if dense:
                self._ddp = nn.parallel.DistributedDataParallel(
                    module, device_ids=[self.device] if self.device.type == "cuda" else None,
                    process_group=self._pg, broadcast_buffers=False, gradient_as_bucket_view=True,
                    static_graph=False)

    # -- torchrec API
    @property
    def module(self) -> nn.Module:
        return self._dmp_wrapped_module

    @module.setter
    def module(self, value: nn.Module) -> None:
        self._dmp_wrapped_module = value

    @property
    def plan(self) -> ShardingPlan:
        return self._plan

    def forward(self, *args, **kwargs):
        if self._ddp is not None:
            return self._ddp(*args, **kwargs)
        return self._dmp_wrapped_module(*args, **kwargs)

    def named_parameters(self, prefix: str = "", recurse: bool = True,
                         remove_duplicate: bool = True) -> Iterator[Tuple[str, nn.Parameter]]:
        yield from self._dmp_wrapped_module.named_parameters(prefix=prefix, recurse=recurse,
                                                             remove_duplicate=remove_duplicate)

    def parameters(self, recurse: bool = True):
        for _, p in self.named_parameters(recurse=recurse):
            yield p

    def state_dict(self, destination=None, prefix: str = "", keep_vars: bool = False):
        return self._dmp_wrapped_module.state_dict(destination=destination, prefix=prefix, keep_vars=keep_vars)

    def load_state_dict(self, state_dict, strict: bool = True):
        return self._dmp_wrapped_module.load_state_dict(state_dict, strict=strict)

    def train(self, mode: bool = True):
        self._dmp_wrapped_module.train(mode)
        self.training = mode
        return self

    def eval(self):
        return self.train(False)


def _is_table_param(root: nn.Module, name: str) -> bool:
    mod_path = name.rsplit(".", 1)[0] if "." in name else ""
    m = root
    parts = mod_path.split(".") if mod_path else []
    chain = [m]
    for p in parts:
        m = getattr(m, p)
        chain.append(m)
    return any(isinstance(x, (EmbeddingBagCollection, ShardedEmbeddingBagCollection)) for x in chain)
