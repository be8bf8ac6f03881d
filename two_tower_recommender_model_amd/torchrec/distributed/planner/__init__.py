"""torchrec.distributed.planner subset: ``EmbeddingShardingPlanner(topology=Topology(...), batch_size,
storage_reservation)`` + ``collective_plan(module, sharders, pg)`` (03_model_training.py:798-811).

The plan is explicit and deterministic (the cost-model search of torchrec's planner is out of
scope): a table larger than half of one rank's fair share of all table bytes is sharded ROW_WISE
over every rank (contiguous row blocks of ceil(N / W)); the others are placed TABLE_WISE greedily
on the rank with the least bytes. ``ParameterConstraints(sharding_types=[...])`` per table name
overrides the choice. World size 1 places everything table-wise on rank 0 unless a constraint says otherwise.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
from torch import nn

from ..types import ParameterSharding, ShardingPlan, ShardingType, ShardMetadata


@dataclass
class Topology:
    world_size: int
    compute_device: str = "cuda"
    hbm_cap: Optional[int] = None
    ddr_cap: Optional[int] = None
    local_world_size: Optional[int] = None
    hbm_mem_bw: Optional[float] = None
    ddr_mem_bw: Optional[float] = None
    intra_host_bw: Optional[float] = None
    inter_host_bw: Optional[float] = None
    bwd_compute_multiplier: Optional[float] = None

    def __post_init__(self):
        if self.local_world_size is None:
            self.local_world_size = self.world_size


@dataclass
class ParameterConstraints:
    sharding_types: Optional[List[str]] = None
    compute_kernels: Optional[List[str]] = None
    min_partition: Optional[int] = None
    pooling_factors: List[float] = field(default_factory=lambda: [1.0])
    num_poolings: Optional[List[float]] = None
    batch_sizes: Optional[List[int]] = None


def _ebc_modules(module: nn.Module):
    from ...modules.embedding_modules import EmbeddingBagCollection

    return [(name, m) for name, m in module.named_modules() if isinstance(m, EmbeddingBagCollection)]


def row_block(num_rows: int, world_size: int) -> int:
    return (num_rows + world_size - 1) // world_size


class EmbeddingShardingPlanner:
    def __init__(self, topology: Optional[Topology] = None, batch_size: Optional[int] = None, enumerator=None,
                 storage_reservation=None, proposer=None, partitioner=None, performance_model=None, stats=None,
                 constraints: Optional[Dict[str, ParameterConstraints]] = None, debug: bool = True):
        if topology is None:
            ws = dist.get_world_size() if dist.is_initialized() else 1
            topology = Topology(world_size=ws, compute_device="cuda")
        self._topology = topology
        self._batch_size = batch_size
        self._storage_reservation = storage_reservation
        self._constraints = constraints or {}

    def plan(self, module: nn.Module, sharders=None) -> ShardingPlan:
        W = self._topology.world_size
        plan = ShardingPlan()
        for path, ebc in _ebc_modules(module):
            cfgs = ebc.embedding_bag_configs()
            tables = {}
            size = {c.name: c.num_embeddings * c.embedding_dim * 4 + c.num_embeddings * 4 for c in cfgs}
            fair_half = sum(size.values()) / max(1, W) / 2
            load = [0] * W
            for c in sorted(cfgs, key=lambda c: (-size[c.name], c.name)):
                forced = self._constraints.get(c.name)
                st = None
                if forced is not None and forced.sharding_types:
                    st = forced.sharding_types[0]
                if st is None and W == 1:
                    st = ShardingType.TABLE_WISE.value
                elif st is None:
                    st = ShardingType.ROW_WISE.value if size[c.name] > fair_half else ShardingType.TABLE_WISE.value
                if st == ShardingType.ROW_WISE.value:
                    bs = row_block(c.num_embeddings, W)
                    spec = []
                    for r in range(W):
                        lo = min(r * bs, c.num_embeddings)
                        n = max(0, min(bs, c.num_embeddings - lo))
                        spec.append(ShardMetadata([lo, 0], [n, c.embedding_dim], f"rank:{r}/cuda:{r}"))
                        load[r] += n * (c.embedding_dim + 1) * 4
                    tables[c.name] = ParameterSharding(st, "fused", list(range(W)), spec)
                elif st == ShardingType.TABLE_WISE.value:
                    r = min(range(W), key=lambda i: (load[i], i))
                    load[r] += size[c.name]
                    spec = [ShardMetadata([0, 0], [c.num_embeddings, c.embedding_dim], f"rank:{r}/cuda:{r}")]
                    tables[c.name] = ParameterSharding(st, "fused", [r], spec)
                else:
                    raise NotImplementedError(f"sharding type {st} is not on the reference's path (TW/RW only)")
            plan.plan[path] = {c.name: tables[c.name] for c in cfgs}
        return plan

    def collective_plan(self, module: nn.Module, sharders=None, pg=None) -> ShardingPlan:
        """Plan on rank 0 and broadcast it (torchrec: broadcast_object_list over the process group)."""
        if pg is None or not dist.is_initialized() or dist.get_world_size() == 1:
            return self.plan(module, sharders)
        obj = [self.plan(module, sharders) if dist.get_rank() == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=pg)
        return obj[0]
