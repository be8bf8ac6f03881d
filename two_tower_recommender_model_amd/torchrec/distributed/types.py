"""torchrec.distributed.types subset: the sharding plan objects printed at
03_model_training.py:818-822 (``model._plan.plan`` -> {module path: {table: ParameterSharding}})."""
from __future__ import annotations

from dataclasses import dataclass, field
from enum import Enum
from typing import Dict, List, Optional


class ShardingType(Enum):
    DATA_PARALLEL = "data_parallel"
    TABLE_WISE = "table_wise"
    ROW_WISE = "row_wise"
    COLUMN_WISE = "column_wise"
    TABLE_ROW_WISE = "table_row_wise"
    TABLE_COLUMN_WISE = "table_column_wise"


class EmbeddingComputeKernel(Enum):
    DENSE = "dense"
    FUSED = "fused"


@dataclass
class ShardMetadata:
    shard_offsets: List[int]
    shard_sizes: List[int]
    placement: str


@dataclass
class ParameterSharding:
    sharding_type: str
    compute_kernel: str
    ranks: Optional[List[int]] = None
    sharding_spec: Optional[List[ShardMetadata]] = None

    def __repr__(self) -> str:
        return (f"ParameterSharding(sharding_type='{self.sharding_type}', compute_kernel='{self.compute_kernel}', "
                f"ranks={self.ranks}, sharding_spec={self.sharding_spec})")


EmbeddingModuleShardingPlan = Dict[str, ParameterSharding]


@dataclass
class ShardingPlan:
    plan: Dict[str, EmbeddingModuleShardingPlan] = field(default_factory=dict)

    def get_plan_for_module(self, module_path: str) -> Optional[EmbeddingModuleShardingPlan]:
        return self.plan.get(module_path)

    def __str__(self) -> str:
        lines = []
        for path, tables in self.plan.items():
            lines.append(f"module: {path}")
            for name, ps in tables.items():
                lines.append(f"  {name}: {ps.sharding_type} ranks={ps.ranks}")
        return "\n".join(lines)
