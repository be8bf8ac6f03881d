"""torchrec.distributed.planner.storage_reservations.HeuristicalStorageReservation (03:806)."""
from __future__ import annotations


class HeuristicalStorageReservation:
    """Fraction of each device's HBM held back from the embedding-table budget."""

    def __init__(self, percentage: float, parameter_multiplier: float = 6.0, dense_tensor_estimate=None):
        if not 0.0 <= percentage <= 1.0:
            raise ValueError("percentage must be in [0, 1]")
        self._percentage = float(percentage)
        self._parameter_multiplier = parameter_multiplier
        self._dense_tensor_estimate = dense_tensor_estimate
