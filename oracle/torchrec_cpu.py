"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — minimal CPU restatement of the torchrec 0.7.0
types the reference's hot-path code touches, so that code can be executed verbatim (by
tests/golden/make_golden.py, in this container only) to produce golden vectors.

Restated semantics (EXTERNAL torchrec 0.7.0, not installed here):
  * KeyedJaggedTensor (sparse/jagged_tensor.py): keys, values, lengths (key-major [F*B]),
    offsets = complete cumsum, stride = B, from_lengths_sync, to_dict, __getitem__.
  * KeyedTensor: values [B, sum D], key -> column slice.
  * EmbeddingBagCollection (modules/embedding_modules.py): one nn.EmbeddingBag(mode="sum",
    include_last_offset=True) per table, features of a table pooled with that table.
  * MLP (modules/mlp.py): Sequential of Perceptron = relu(Linear(x)) on every layer, stored at
    ``_mlp[i]._linear``.
  * Batch (datasets/utils.py): dense_features, sparse_features, labels.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F
from torch import nn


class KeyedJaggedTensor:
    def __init__(self, keys: List[str], values: torch.Tensor, lengths: torch.Tensor,
                 stride: Optional[int] = None):
        self._keys = list(keys)
        self._values = values
        self._lengths = lengths
        self._stride = stride if stride is not None else (lengths.numel() // max(1, len(keys)))
        self._offsets = torch.cat([torch.zeros(1, dtype=lengths.dtype), torch.cumsum(lengths, 0).to(lengths.dtype)])

    @staticmethod
    def from_lengths_sync(keys, values, lengths, weights=None, stride=None):
        return KeyedJaggedTensor(keys, values, lengths, stride)

    def keys(self):
        return self._keys

    def values(self):
        return self._values

    def lengths(self):
        return self._lengths

    def offsets(self):
        return self._offsets

    def stride(self):
        return self._stride

    def length_per_key(self):
        B = self._stride
        return [int(self._lengths[i * B:(i + 1) * B].sum()) for i in range(len(self._keys))]


@dataclass
class KeyedTensor:
    keys: List[str]
    length_per_key: List[int]
    values: torch.Tensor

    def __getitem__(self, key: str) -> torch.Tensor:
        i = self.keys.index(key)
        s = sum(self.length_per_key[:i])
        return self.values[:, s:s + self.length_per_key[i]]


@dataclass
class Batch:
    dense_features: torch.Tensor
    sparse_features: KeyedJaggedTensor
    labels: torch.Tensor


@dataclass
class EmbeddingBagConfig:
    num_embeddings: int
    embedding_dim: int
    name: str = ""
    feature_names: List[str] = field(default_factory=list)


class EmbeddingBagCollection(nn.Module):
    def __init__(self, tables: List[EmbeddingBagConfig], device=None):
        super().__init__()
        self._configs = tables
        self.embedding_bags = nn.ModuleDict({
            t.name: nn.EmbeddingBag(t.num_embeddings, t.embedding_dim, mode="sum", include_last_offset=True)
            for t in tables
        })

    def embedding_bag_configs(self):
        return self._configs

    def forward(self, kjt: KeyedJaggedTensor) -> KeyedTensor:
        B = kjt.stride()
        keys = kjt.keys()
        offs = kjt.offsets().to(torch.int64)
        outs, names, dims = [], [], []
        for cfg in self._configs:
            for fname in cfg.feature_names:
                f = keys.index(fname)
                s, e = int(offs[f * B]), int(offs[(f + 1) * B])
                idx = kjt.values()[s:e].to(torch.int64)
                off = offs[f * B:(f + 1) * B + 1] - s
                outs.append(self.embedding_bags[cfg.name](idx, off).float())
                names.append(fname)
                dims.append(cfg.embedding_dim)
        return KeyedTensor(names, dims, torch.cat(outs, dim=1))


class Perceptron(nn.Module):
    def __init__(self, in_size, out_size, bias=True, activation=torch.relu, device=None):
        super().__init__()
        self._linear = nn.Linear(in_size, out_size, bias=bias, device=device)
        self._activation_fn = activation

    def forward(self, x):
        return self._activation_fn(self._linear(x))


class MLP(nn.Module):
    def __init__(self, in_size, layer_sizes, bias=True, activation=torch.relu, device=None):
        super().__init__()
        self._mlp = nn.Sequential(*[
            Perceptron(layer_sizes[i - 1] if i > 0 else in_size, layer_sizes[i], bias, activation)
            for i in range(len(layer_sizes))
        ])

    def forward(self, x):
        return self._mlp(x)
