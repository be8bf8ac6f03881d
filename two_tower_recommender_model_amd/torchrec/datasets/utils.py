"""torchrec.datasets.utils.Batch — the container built by transform_to_torchrec_batch
(03_model_training.py:376-380) and moved to the device by the pipeline."""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ..sparse.jagged_tensor import KeyedJaggedTensor


@dataclass
class Batch:
    dense_features: torch.Tensor
    sparse_features: KeyedJaggedTensor
    labels: torch.Tensor

    def to(self, device: torch.device, non_blocking: bool = False) -> "Batch":
        return Batch(
            dense_features=self.dense_features.to(device=device, non_blocking=non_blocking),
            sparse_features=self.sparse_features.to(device=device, non_blocking=non_blocking),
            labels=self.labels.to(device=device, non_blocking=non_blocking),
        )

    def record_stream(self, stream) -> None:
        if self.dense_features.is_cuda:
            self.dense_features.record_stream(stream)
        self.sparse_features.record_stream(stream)
        if self.labels.is_cuda:
            self.labels.record_stream(stream)

    def pin_memory(self) -> "Batch":
        return Batch(self.dense_features.pin_memory(), self.sparse_features.pin_memory(), self.labels.pin_memory())
