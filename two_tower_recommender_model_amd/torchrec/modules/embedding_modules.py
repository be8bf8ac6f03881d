"""torchrec.modules.embedding_modules.EmbeddingBagCollection on the MI355X kernels.

API as used by the reference: ``EmbeddingBagCollection(tables=eb_configs, device=...)``
(03_model_training.py:781-784), ``.embedding_bag_configs()`` (:404-410), ``forward(kjt) ->
KeyedTensor`` (:417), state-dict keys ``embedding_bags.<table>.weight`` (:1030 reload path).

Storage: all tables of the collection live in ONE flat fp32 HBM buffer (``ops.TableSet``: per-table
element offsets, FBGEMM-TBE style) with the row-wise optimizer state beside it; each
``embedding_bags[name].weight`` Parameter is a view into it. Forward = one ``tt_pooled_fwd`` launch
for every key of the KJT writing the [B, sum D] KeyedTensor directly. Backward, when the tables
carry ``_apply_optimizer_in_backward(RowWiseAdagrad, ...)`` (03:791-795): the dedup +
fused row-wise Adagrad kernels update the weights in place and the Parameters' ``.grad`` stays
None (what FBGEMM's fused TBE does); otherwise a dense gradient is produced for the optimizer the
user attached.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
from torch import nn

from ... import _lib, ops
from ..sparse.jagged_tensor import KeyedJaggedTensor, KeyedTensor
from .embedding_configs import EmbeddingBagConfig, PoolingType


class _TableModule(nn.Module):
    """Holds ``weight`` so the state-dict key is ``embedding_bags.<name>.weight`` (as nn.EmbeddingBag)."""

    def __init__(self, weight: nn.Parameter):
        super().__init__()
        self.weight = weight


def _fused_config(params: List[nn.Parameter]) -> Optional[Dict[str, float]]:
    """Read the optimizer torch's _apply_optimizer_in_backward attached to the table params. Returns
    the fused row-wise Adagrad hyper-parameters, or None (dense gradient path)."""
    cfg = None
    for p in params:
        classes = getattr(p, "_optimizer_classes", None)
        kwargs = getattr(p, "_optimizer_kwargs", None)
        if not classes:
            return None
        cls, kw = classes[-1], dict(kwargs[-1])
        if getattr(cls, "__name__", "") != "RowWiseAdagrad":
            return None
        if float(kw.get("weight_decay", 0.0)) != 0.0 or float(kw.get("lr_decay", 0.0)) != 0.0:
            return None
        if float(kw.get("initial_accumulator_value", 0.0)) != 0.0:
            return None
        c = {"lr": float(kw.get("lr", 1e-2)), "eps": float(kw.get("eps", 1e-10))}
        if cfg is not None and cfg != c:
            raise _lib.TTError("tables of one EmbeddingBagCollection must share the in-backward optimizer config")
        cfg = c
    return cfg


class _PooledLookup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ebc, ts, values, offsets, B, pooling, *weights):
        out = ts.pooled_fwd(values, offsets, B, pooling=pooling)
        ctx.ebc = ebc
        ctx.ts = ts
        ctx.B = B
        ctx.pooling = pooling
        ctx.save_for_backward(values, offsets)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        values, offsets = ctx.saved_tensors
        ebc = ctx.ebc
        ts = ctx.ts
        B = ctx.B
        if grad_out.stride(1) != 1 or grad_out.stride(0) != grad_out.shape[1]:
            grad_out = grad_out.contiguous()
        nw = len(ebc._params())
        fused = ebc._fused_cfg()
        if fused is not None:
            ts.bwd_prepare(values, offsets, B, max_lookups=max(1, values.numel()))
            ts.bwd_rowwise_adagrad(grad_out, offsets, B, fused["lr"], fused["eps"], pooling=ctx.pooling)
            return (None,) * 6 + (None,) * nw
        gw = torch.zeros_like(ts.weights)
        ts.bwd_dense(grad_out, values, offsets, B, gw, pooling=ctx.pooling)
        grads = []
        for t in range(ts.T):
            o = ts.weight_offsets[t]
            grads.append(gw[o:o + ts.rows[t] * ts.dims[t]].view(ts.rows[t], ts.dims[t]))
        return (None,) * 6 + tuple(grads)


class EmbeddingBagCollection(nn.Module):
    def __init__(self, tables: List[EmbeddingBagConfig], is_weighted: bool = False,
                 device: Optional[torch.device] = None):
        super().__init__()
        if is_weighted:
            raise NotImplementedError("weighted KJTs are not on the reference's path")
        self._is_weighted = is_weighted
        self._embedding_bag_configs = list(tables)
        names = [t.name for t in tables]
        if len(set(names)) != len(names):
            raise ValueError("duplicate table names")
        pools = {t.pooling for t in tables}
        if len(pools) != 1 or PoolingType.NONE in pools:
            raise NotImplementedError("one of SUM / MEAN pooling for all tables is supported")
        self._pooling = _lib.TT_POOL_MEAN if PoolingType.MEAN in pools else _lib.TT_POOL_SUM
        self._feature_names: List[str] = []
        self._feature_table: List[int] = []
        self._lengths_per_embedding: List[int] = []
        for t_idx, t in enumerate(tables):
            for f in t.feature_names:
                self._feature_names.append(f)
                self._feature_table.append(t_idx)
                self._lengths_per_embedding.append(t.embedding_dim)
        self._embedding_names = list(self._feature_names)
        device = torch.device(device) if device is not None else torch.device("cpu")
        self.embedding_bags = nn.ModuleDict()
        self._ts: Optional[ops.TableSet] = None
        self._meta_cache: Dict[Tuple[str, ...], ops.TableSet] = {}
        if device.type == "cuda":
            self._materialize(device)
        else:
            for t in tables:
                w = torch.empty(t.num_embeddings, t.embedding_dim, device=device)
                if device.type != "meta":
                    w.uniform_(t.get_weight_init_min(), t.get_weight_init_max())
                self.embedding_bags[t.name] = _TableModule(nn.Parameter(w))

    # -- torchrec API
    def embedding_bag_configs(self) -> List[EmbeddingBagConfig]:
        return self._embedding_bag_configs

    def is_weighted(self) -> bool:
        return self._is_weighted

    @property
    def device(self) -> torch.device:
        return self._params()[0].device if self._params() else torch.device("cpu")

    # -- storage
    def _params(self) -> List[nn.Parameter]:
        return [self.embedding_bags[t.name].weight for t in self._embedding_bag_configs
                if t.name in self.embedding_bags]

    def _fused_cfg(self) -> Optional[Dict[str, float]]:
        return _fused_config(self._params())

    def _bound_to_ts(self) -> bool:
        if self._ts is None:
            return False
        for t, p in enumerate(self._params()):
            if p.device != self._ts.device or p.data_ptr() != self._ts.table_view(t).data_ptr():
                return False
        return True

    def _materialize(self, device: torch.device, init: str = "auto") -> None:
        """(Re)bind every table Parameter to a view of one flat HBM buffer. Existing (non-meta)
        values are copied; meta tables get torchrec's default init U(-sqrt(1/N), sqrt(1/N))."""
        tables = self._embedding_bag_configs
        old = {t.name: self.embedding_bags[t.name].weight for t in tables if t.name in self.embedding_bags}
        ts = ops.TableSet([t.num_embeddings for t in tables], [t.embedding_dim for t in tables],
                          self._feature_table, device)
        for ti, t in enumerate(tables):
            view = ts.table_view(ti)
            src = old.get(t.name)
            if src is not None and src.device.type != "meta" and init != "random":
                view.copy_(src.detach())
            else:
                view.uniform_(t.get_weight_init_min(), t.get_weight_init_max())
            p = nn.Parameter(view)
            if src is not None:
                for cls, kw in zip(getattr(src, "_optimizer_classes", []), getattr(src, "_optimizer_kwargs", [])):
                    # re-attach the in-backward optimizer to the new Parameter
                    from torch.distributed.optim import _apply_optimizer_in_backward
                    _apply_optimizer_in_backward(cls, [p], kw)
            self.embedding_bags[t.name] = _TableModule(p)
        self._ts = ts
        self._meta_cache = {}

    def _table_set_for_keys(self, keys: List[str]) -> Tuple[ops.TableSet, Optional[List[int]]]:
        """TableSet whose feature map follows the KJT's key order (no copy); or a key permutation
        to apply first when the KJT carries keys this collection does not own."""
        feats = self._feature_names
        if list(keys) == feats:
            return self._ts, None
        if sorted(keys) == sorted(feats):
            k = tuple(keys)
            ts = self._meta_cache.get(k)
            if ts is None:
                col, o = {}, 0
                for f, d in zip(feats, self._lengths_per_embedding):
                    col[f] = o
                    o += d
                ts = self._ts.remap([self._feature_table[feats.index(n)] for n in keys], [col[n] for n in keys])
                self._meta_cache[k] = ts
            return ts, None
        missing = [f for f in feats if f not in keys]
        if missing:
            raise KeyError(f"KJT lacks features {missing}")
        return self._ts, [list(keys).index(f) for f in feats]

    def forward(self, features: KeyedJaggedTensor) -> KeyedTensor:
        if not features.values().is_cuda and features.values().numel() > 0:
            raise _lib.TTError("EmbeddingBagCollection runs on the MI355X kernels only: move the KJT to the GPU")
        dev = features.lengths().device
        if not self._bound_to_ts() or self._ts.device != dev:
            self._materialize(dev)
        ts, perm = self._table_set_for_keys(features.keys())
        if perm is not None:
            features = features.permute(perm)
        B = features.stride()
        values = features.values()
        if values.dtype not in (torch.int32, torch.int64):
            if values.numel() != 0:
                raise _lib.TTError("KJT values must be int32/int64 ids")
            values = values.to(torch.int64)  # the reference's all-zero batch gives an empty float tensor
        offsets = features.offsets()
        if offsets.dtype != torch.int32:
            offsets = offsets.to(torch.int32)
        pooled = _PooledLookup.apply(self, ts, values, offsets, B, self._pooling, *self._params())
        return KeyedTensor(self._embedding_names, self._lengths_per_embedding, pooled)
