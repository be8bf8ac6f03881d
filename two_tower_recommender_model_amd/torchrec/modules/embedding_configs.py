"""torchrec.modules.embedding_configs — EmbeddingBagConfig as constructed at
03_model_training.py:770-778 (name, embedding_dim, num_embeddings, feature_names)."""
from __future__ import annotations

from dataclasses import dataclass, field
from enum import Enum, unique
from typing import List, Optional


@unique
class PoolingType(Enum):
    SUM = "SUM"
    MEAN = "MEAN"
    NONE = "NONE"


@unique
class DataType(Enum):
    FP32 = "FP32"
    FP16 = "FP16"
    BF16 = "BF16"
    INT64 = "INT64"
    INT32 = "INT32"


@dataclass
class BaseEmbeddingConfig:
    num_embeddings: int
    embedding_dim: int
    name: str = ""
    data_type: DataType = DataType.FP32
    feature_names: List[str] = field(default_factory=list)
    weight_init_max: Optional[float] = None
    weight_init_min: Optional[float] = None
    num_embeddings_post_pruning: Optional[int] = None
    init_fn: Optional[object] = None
    need_pos: bool = False

    def get_weight_init_max(self) -> float:
        return self.weight_init_max if self.weight_init_max is not None else (1.0 / self.num_embeddings) ** 0.5

    def get_weight_init_min(self) -> float:
        return self.weight_init_min if self.weight_init_min is not None else -((1.0 / self.num_embeddings) ** 0.5)

    def num_features(self) -> int:
        return len(self.feature_names)


@dataclass
class EmbeddingBagConfig(BaseEmbeddingConfig):
    pooling: PoolingType = PoolingType.SUM


@dataclass
class EmbeddingConfig(BaseEmbeddingConfig):
    pass
