"""KeyedJaggedTensor / KeyedTensor — the torchrec.sparse.jagged_tensor API the reference uses
(03_model_training.py:367-371 ``from_lengths_sync``; :417-436 ``pooled_embeddings[feature]``;
:1081-1091 ctor with keys/values/lengths).

Layout (torchrec 0.7.0): ``keys[F]``, ``values[sum L]``, ``lengths[F*B]`` key-major,
``offsets = [0, cumsum(lengths)]``, ``stride() = B``. On a device the offsets come from the HIP
complete-cumsum kernel; on the host (batches built by the data loader before H2D) from torch.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from ... import ops


def _offsets_from_lengths(lengths: torch.Tensor) -> torch.Tensor:
    if lengths.is_cuda:
        return ops.complete_cumsum(lengths.to(torch.int32))
    out = torch.zeros(lengths.numel() + 1, dtype=torch.int64)
    torch.cumsum(lengths.to(torch.int64), 0, out=out[1:])
    return out.to(lengths.dtype if lengths.dtype in (torch.int32, torch.int64) else torch.int32)


class JaggedTensor:
    def __init__(self, values: torch.Tensor, lengths: torch.Tensor, offsets: Optional[torch.Tensor] = None,
                 weights: Optional[torch.Tensor] = None):
        self._values = values
        self._lengths = lengths
        self._offsets = offsets
        self._weights = weights

    def values(self):
        return self._values

    def lengths(self):
        return self._lengths

    def offsets(self):
        if self._offsets is None:
            self._offsets = _offsets_from_lengths(self._lengths)
        return self._offsets

    def weights_or_none(self):
        return self._weights

    def to_dense(self) -> List[torch.Tensor]:
        o = self.offsets().tolist()
        return [self._values[o[i]:o[i + 1]] for i in range(len(o) - 1)]


class KeyedJaggedTensor:
    def __init__(self, keys: List[str], values: torch.Tensor, weights: Optional[torch.Tensor] = None,
                 lengths: Optional[torch.Tensor] = None, offsets: Optional[torch.Tensor] = None,
                 stride: Optional[int] = None, length_per_key: Optional[List[int]] = None,
                 offset_per_key: Optional[List[int]] = None, index_per_key=None, jt_dict=None,
                 inverse_indices=None):
        self._keys = list(keys)
        self._values = values
        self._weights = weights
        if lengths is None and offsets is None:
            raise ValueError("KeyedJaggedTensor needs lengths or offsets")
        if lengths is None:
            lengths = (offsets[1:] - offsets[:-1]).to(torch.int32)
        self._lengths = lengths
        self._offsets = offsets
        if stride is None:
            stride = lengths.numel() // len(self._keys) if self._keys else 0
        self._stride = int(stride)
        self._length_per_key = length_per_key
        self._offset_per_key = offset_per_key

    # -- constructors (torchrec names)
    @staticmethod
    def from_lengths_sync(keys: List[str], values: torch.Tensor, lengths: torch.Tensor,
                          weights: Optional[torch.Tensor] = None, stride: Optional[int] = None) -> "KeyedJaggedTensor":
        kjt = KeyedJaggedTensor(keys=keys, values=values, weights=weights, lengths=lengths, stride=stride)
        kjt.sync()
        return kjt

    @staticmethod
    def from_offsets_sync(keys: List[str], values: torch.Tensor, offsets: torch.Tensor,
                          weights: Optional[torch.Tensor] = None, stride: Optional[int] = None) -> "KeyedJaggedTensor":
        kjt = KeyedJaggedTensor(keys=keys, values=values, weights=weights, offsets=offsets, stride=stride)
        kjt.sync()
        return kjt

    @staticmethod
    def empty(is_weighted: bool = False, device=None, values_dtype=None, weights_dtype=None,
              lengths_dtype=torch.int32) -> "KeyedJaggedTensor":
        v = torch.empty(0, dtype=values_dtype or torch.int64, device=device)
        return KeyedJaggedTensor([], v, weights=(torch.empty(0, device=device) if is_weighted else None),
                                 lengths=torch.empty(0, dtype=lengths_dtype, device=device), stride=0)

    # -- accessors
    def sync(self) -> "KeyedJaggedTensor":
        self.length_per_key()
        return self

    def keys(self) -> List[str]:
        return self._keys

    def values(self) -> torch.Tensor:
        return self._values

    def weights(self) -> torch.Tensor:
        if self._weights is None:
            raise ValueError("KeyedJaggedTensor is unweighted")
        return self._weights

    def weights_or_none(self) -> Optional[torch.Tensor]:
        return self._weights

    def lengths(self) -> torch.Tensor:
        return self._lengths

    def offsets(self) -> torch.Tensor:
        if self._offsets is None:
            self._offsets = _offsets_from_lengths(self._lengths)
        return self._offsets

    def stride(self) -> int:
        return self._stride

    def device(self) -> torch.device:
        return self._values.device

    def length_per_key(self) -> List[int]:
        if self._length_per_key is None:
            B = self._stride
            o = self.offsets()
            idx = torch.arange(0, len(self._keys) + 1, device=o.device) * B
            b = o[idx].to(torch.int64).cpu().tolist()  # host sync (as torchrec's *_sync)
            self._length_per_key = [b[i + 1] - b[i] for i in range(len(self._keys))]
        return self._length_per_key

    def offset_per_key(self) -> List[int]:
        if self._offset_per_key is None:
            acc, out = 0, [0]
            for n in self.length_per_key():
                acc += n
                out.append(acc)
            self._offset_per_key = out
        return self._offset_per_key

    def to_dict(self) -> Dict[str, JaggedTensor]:
        B = self._stride
        opk = self.offset_per_key()
        out = {}
        for i, k in enumerate(self._keys):
            s, e = opk[i], opk[i + 1]
            w = self._weights[s:e] if self._weights is not None else None
            out[k] = JaggedTensor(self._values[s:e], self._lengths[i * B:(i + 1) * B], weights=w)
        return out

    def __getitem__(self, key: str) -> JaggedTensor:
        return self.to_dict()[key]

    # -- transforms
    def permute(self, indices: List[int], indices_tensor: Optional[torch.Tensor] = None) -> "KeyedJaggedTensor":
        """KJT.permute -> permute_2D_sparse_data (HIP kernel on device tensors)."""
        B = self._stride
        keys = [self._keys[i] for i in indices]
        if self._values.is_cuda:
            lpk = self.length_per_key()
            total = sum(lpk[i] for i in indices)
            lengths, offsets, values, weights = ops.kjt_permute(
                self._lengths.to(torch.int32), self.offsets().to(torch.int32), self._values, len(self._keys), B,
                indices, weights=self._weights, total=total)
            return KeyedJaggedTensor(keys, values, weights=weights, lengths=lengths, offsets=offsets, stride=B,
                                     length_per_key=[lpk[i] for i in indices])
        opk = self.offset_per_key()
        lens = torch.cat([self._lengths[i * B:(i + 1) * B] for i in indices]) if indices else self._lengths[:0]
        vals = torch.cat([self._values[opk[i]:opk[i + 1]] for i in indices]) if indices else self._values[:0]
        w = None
        if self._weights is not None:
            w = torch.cat([self._weights[opk[i]:opk[i + 1]] for i in indices]) if indices else self._weights[:0]
        return KeyedJaggedTensor(keys, vals, weights=w, lengths=lens, stride=B)

    def split(self, segments: List[int]) -> List["KeyedJaggedTensor"]:
        out, k = [], 0
        for seg in segments:
            out.append(self.permute(list(range(k, k + seg))))
            k += seg
        return out

    def to(self, device: torch.device, non_blocking: bool = False, dtype=None) -> "KeyedJaggedTensor":
        w = self._weights.to(device, non_blocking=non_blocking) if self._weights is not None else None
        o = self._offsets.to(device, non_blocking=non_blocking) if self._offsets is not None else None
        return KeyedJaggedTensor(self._keys, self._values.to(device, non_blocking=non_blocking), weights=w,
                                 lengths=self._lengths.to(device, non_blocking=non_blocking), offsets=o,
                                 stride=self._stride, length_per_key=self._length_per_key,
                                 offset_per_key=self._offset_per_key)

    def pin_memory(self) -> "KeyedJaggedTensor":
        w = self._weights.pin_memory() if self._weights is not None else None
        o = self._offsets.pin_memory() if self._offsets is not None else None
        return KeyedJaggedTensor(self._keys, self._values.pin_memory(), weights=w,
                                 lengths=self._lengths.pin_memory(), offsets=o, stride=self._stride,
                                 length_per_key=self._length_per_key, offset_per_key=self._offset_per_key)

    def record_stream(self, stream) -> None:
        for t in (self._values, self._lengths, self._offsets, self._weights):
            if t is not None and t.is_cuda:
                t.record_stream(stream)

    def __repr__(self) -> str:
        return (f"KeyedJaggedTensor(keys={self._keys}, stride={self._stride}, "
                f"values={tuple(self._values.shape)}:{self._values.dtype})")


class KeyedTensor:
    """Pooled embeddings: values [B, sum D] (key_dim 1), ``kt[key]`` is a column-slice view."""

    def __init__(self, keys: List[str], length_per_key: List[int], values: torch.Tensor, key_dim: int = 1):
        self._keys = list(keys)
        self._length_per_key = list(length_per_key)
        self._values = values
        self._key_dim = key_dim
        self._offset_per_key = [0]
        for n in self._length_per_key:
            self._offset_per_key.append(self._offset_per_key[-1] + n)
        self._index = {k: i for i, k in enumerate(self._keys)}

    def keys(self) -> List[str]:
        return self._keys

    def values(self) -> torch.Tensor:
        return self._values

    def length_per_key(self) -> List[int]:
        return self._length_per_key

    def offset_per_key(self) -> List[int]:
        return self._offset_per_key

    def key_dim(self) -> int:
        return self._key_dim

    def __getitem__(self, key: str) -> torch.Tensor:
        i = self._index[key]
        return self._values[:, self._offset_per_key[i]:self._offset_per_key[i + 1]]

    def to_dict(self) -> Dict[str, torch.Tensor]:
        return {k: self[k] for k in self._keys}

    def record_stream(self, stream) -> None:
        if self._values.is_cuda:
            self._values.record_stream(stream)
