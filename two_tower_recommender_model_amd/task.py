"""TwoTower + TwoTowerTrainTask with the reference's semantics (03_model_training.py:395-455),
generalised to several features per tower (the ray-tune variant's concatenation,
ray_tune_optuna_tuning_alex_test.py:270-306), on the MI355X kernels.

  q = MLP_query(cat(kt[f] for f in query features)); c = MLP_cand(cat(...))
  logits = (q * c).sum(1).squeeze(); loss = BCEWithLogits(mean)

Differences from running the reference's classes on the torchrec shim (which also works): tower
inputs that are adjacent KeyedTensor columns are passed as views (no torch.cat copy), and the dot
+ BCE + its gradient is one HIP kernel (k5) instead of five torch ops.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
from torch import nn

from . import ops
from .torchrec.datasets.utils import Batch
from .torchrec.modules.embedding_modules import EmbeddingBagCollection
from .torchrec.modules.mlp import MLP


class _DotBCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, c, labels, kernel):
        B, d = q.shape
        q = q.contiguous()
        c = c.contiguous()
        dq = torch.empty_like(q)
        dc = torch.empty_like(c)
        logits, loss = kernel(q, c, labels, dq=dq, dc=dc)
        ctx.save_for_backward(dq, dc)
        ctx.mark_non_differentiable(logits)
        return loss, logits

    @staticmethod
    def backward(ctx, gloss, glogits):
        dq, dc = ctx.saved_tensors
        # d(loss)/dq precomputed with grad_scale 1; chain the upstream scalar gradient
        return dq * gloss, dc * gloss, None, None


def _tower_input(kt, names: Sequence[str]) -> torch.Tensor:
    keys = kt.keys()
    idx = [keys.index(n) for n in names]
    if idx == list(range(idx[0], idx[0] + len(idx))):
        opk = kt.offset_per_key()
        return kt.values()[:, opk[idx[0]]:opk[idx[-1] + 1]]
    return torch.cat([kt[n] for n in names], dim=1)


class TwoTower(nn.Module):
    def __init__(self, embedding_bag_collection: EmbeddingBagCollection, layer_sizes: List[int],
                 query_features: Optional[List[str]] = None, candidate_features: Optional[List[str]] = None,
                 device: Optional[torch.device] = None):
        super().__init__()
        cfgs = embedding_bag_collection.embedding_bag_configs()
        if query_features is None or candidate_features is None:
            # the reference: table 0 = query tower, table 1 = candidate tower (03:404-410)
            assert len(cfgs) == 2, "Expected two EmbeddingBags in the two tower model"
            query_features = list(cfgs[0].feature_names)
            candidate_features = list(cfgs[1].feature_names)
        dim = {f: c.embedding_dim for c in cfgs for f in c.feature_names}
        self._feature_names_query = list(query_features)
        self._candidate_feature_names = list(candidate_features)
        self.ebc = embedding_bag_collection
        self.query_proj = MLP(in_size=sum(dim[f] for f in query_features), layer_sizes=layer_sizes, device=device)
        self.candidate_proj = MLP(in_size=sum(dim[f] for f in candidate_features), layer_sizes=layer_sizes,
                                  device=device)

    def forward(self, kjt) -> Tuple[torch.Tensor, torch.Tensor]:
        kt = self.ebc(kjt)
        q = self.query_proj(_tower_input(kt, self._feature_names_query))
        c = self.candidate_proj(_tower_input(kt, self._candidate_feature_names))
        return q, c


class TwoTowerTrainTask(nn.Module):
    def __init__(self, two_tower: TwoTower, max_batch: int = 1 << 16) -> None:
        super().__init__()
        self.two_tower = two_tower
        self._max_batch = max_batch
        self._k = None

    def forward(self, batch: Batch):
        q, c = self.two_tower(batch.sparse_features)
        if q.shape[0] == 1:
            # the reference squeezes the [1] logits to 0-d (03_model_training.py:452) and
            # BCEWithLogitsLoss then rejects the [1] labels: a batch of one cannot train there
            raise ValueError(f"Target size ({batch.labels.shape}) must be the same as input size (torch.Size([]))")
        if self._k is None or self._k.device != q.device or self._k.max_batch < q.shape[0]:
            self._k = ops.DotBCE(q.device, max(self._max_batch, q.shape[0]))
        loss, logits = _DotBCE.apply(q, c, batch.labels, self._k)
        logits = logits.squeeze()
        return loss, (loss.detach(), logits.detach(), batch.labels.detach())
