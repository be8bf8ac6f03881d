"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — CPU restatement of the two-tower hot path.

Integer/byte work is numpy; floating point follows TorchRec's unsharded CPU arithmetic with torch on
the CPU (``F.embedding_bag`` is exactly what torchrec's CPU ``EmbeddingBagCollection`` calls). Every
function cites the reference file:line (or the pinned third-party algorithm) it restates.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

# ----------------------------------------------------------------------------------------------
# a1: KJT build — transform_to_torchrec_batch, 03_model_training.py:353-382
# ----------------------------------------------------------------------------------------------


def kjt_build(cols: Sequence[np.ndarray], num_embeddings: Sequence[int]):
    """Column-major walk over cat_cols (03:356); id kept iff truthy (03:358), value = id % N
    (Python floor-mod, 03:360), length 1 else 0 (03:362-365). Returns (values, lengths int32,
    offsets int32). values keep the column dtype; an all-dropped batch yields float32 (what
    ``torch.tensor([])`` gives at 03:369)."""
    vals, lens = [], []
    for c, n in zip(cols, num_embeddings):
        c = np.asarray(c)
        keep = c != 0
        lens.append(keep.astype(np.int32))
        vals.append(np.mod(c[keep], np.asarray(n, dtype=c.dtype)).astype(c.dtype))
    lengths = np.concatenate(lens) if lens else np.zeros(0, np.int32)
    values = np.concatenate(vals) if vals else np.zeros(0, np.float32)
    if values.size == 0:
        values = np.zeros(0, np.float32)
    return values, lengths, complete_cumsum(lengths)


def complete_cumsum(lengths: np.ndarray) -> np.ndarray:
    """fbgemm asynchronous_complete_cumsum: [0, cumsum(lengths)] (KJT offsets)."""
    out = np.zeros(lengths.size + 1, np.int64)
    np.cumsum(lengths, out=out[1:])
    return out.astype(np.int32)


def kjt_permute(lengths: np.ndarray, values: np.ndarray, F_: int, B: int, perm: Sequence[int],
                weights: Optional[np.ndarray] = None):
    """fbgemm permute_2D_sparse_data / KeyedJaggedTensor.permute: key segments reordered."""
    offs = complete_cumsum(lengths).astype(np.int64)
    out_l, out_v, out_w = [], [], []
    for p in perm:
        out_l.append(lengths[p * B:(p + 1) * B])
        s, e = offs[p * B], offs[(p + 1) * B]
        out_v.append(values[s:e])
        if weights is not None:
            out_w.append(weights[s:e])
    ol = np.concatenate(out_l) if out_l else np.zeros(0, lengths.dtype)
    ov = np.concatenate(out_v) if out_v else values[:0]
    ow = (np.concatenate(out_w) if out_w else weights[:0]) if weights is not None else None
    return ol, ov, ow


def block_bucketize(lengths: np.ndarray, values: np.ndarray, F_: int, B: int,
                    block_sizes: Sequence[int], W: int):
    """fbgemm block_bucketize_sparse_features (keep_orig_idx=False, no pos/sequence):
    p = id // bs if id < bs*W else id % W; local = id % bs if id < bs*W else id // W.
    Output bucket-major [W][F][B]; inside one (bucket, bag) ids keep input order."""
    offs = complete_cumsum(lengths).astype(np.int64)
    new_len = np.zeros((W, F_ * B), np.int32)
    buckets: List[List[List[int]]] = [[[] for _ in range(F_ * B)] for _ in range(W)]
    for i in range(F_ * B):
        f = i // B
        bs = int(block_sizes[f])
        for j in range(offs[i], offs[i + 1]):
            idv = int(values[j])
            if idv < bs * W:
                p, loc = idv // bs, idv % bs
            else:
                p, loc = idv % W, idv // W
            buckets[p][i].append(loc)
            new_len[p, i] += 1
    new_vals = [v for p in range(W) for i in range(F_ * B) for v in buckets[p][i]]
    return new_len.reshape(-1), np.asarray(new_vals, dtype=values.dtype)


# ----------------------------------------------------------------------------------------------
# a4: EBC sum pooling — torchrec EmbeddingBagCollection.forward (unsharded CPU): one
# nn.EmbeddingBag(mode="sum", include_last_offset=True) per table (self.ebc(kjt), 03:417)
# ----------------------------------------------------------------------------------------------


def pooled_fwd(tables: Sequence[torch.Tensor], feature_table: Sequence[int], values: torch.Tensor,
               offsets: torch.Tensor, B: int, pooling: str = "sum") -> torch.Tensor:
    """KeyedTensor values [B, sum D] in feature order."""
    outs = []
    offsets = offsets.to(torch.int64)
    for f, t in enumerate(feature_table):
        s, e = int(offsets[f * B]), int(offsets[(f + 1) * B])
        idx = values[s:e].to(torch.int64)
        off = offsets[f * B:(f + 1) * B + 1] - s
        outs.append(F.embedding_bag(idx, tables[t], off, mode=pooling, include_last_offset=True))
    return torch.cat(outs, dim=1) if outs else torch.zeros(B, 0)


def pooled_bwd_dense(tables: Sequence[torch.Tensor], feature_table: Sequence[int],
                     values: torch.Tensor, offsets: torch.Tensor, B: int, grad_out: torch.Tensor,
                     pooling: str = "sum") -> List[torch.Tensor]:
    """Dense table gradients of pooled_fwd (nn.EmbeddingBag dense backward = index_add,
    duplicates summed)."""
    ts = [t.detach().clone().requires_grad_(True) for t in tables]
    out = pooled_fwd(ts, feature_table, values, offsets, B, pooling)
    out.backward(grad_out)
    return [t.grad if t.grad is not None else torch.zeros_like(t) for t in ts]


# ----------------------------------------------------------------------------------------------
# a8: torchrec RowWiseAdagrad (lr=1e-2 default, eps=1e-10, lr_decay=weight_decay=0, init 0),
# applied in backward via _apply_optimizer_in_backward (03_model_training.py:791-795)
# ----------------------------------------------------------------------------------------------


def rowwise_adagrad(weight: torch.Tensor, state: torch.Tensor, grad: torch.Tensor, lr: float,
                    eps: float = 1e-10) -> None:
    """In place: state[r] += mean_d grad[r,d]^2; weight += -lr * grad / (sqrt(state) + eps).
    state is [N] (torchrec keeps [N, 1]). Rows with zero grad are unchanged (identical to the
    dense update, which adds 0)."""
    row = grad.pow(2).mean(dim=1)
    state.add_(row)
    std = state.sqrt().add_(eps).view(-1, 1)
    weight.addcdiv_(grad, std, value=-lr)


def rowwise_adagrad_sparse(weight: torch.Tensor, state: torch.Tensor, rows: torch.Tensor,
                           grad_rows: torch.Tensor, lr: float, eps: float = 1e-10) -> None:
    """The same update restricted to the unique touched rows (mathematically identical)."""
    sub_w = weight[rows]
    sub_s = state[rows]
    rowwise_adagrad(sub_w, sub_s, grad_rows, lr, eps)
    weight[rows] = sub_w
    state[rows] = sub_s


# ----------------------------------------------------------------------------------------------
# a6/a7: torchrec MLP (Perceptron = Linear + ReLU on every layer, 03:411-412) and the task head
# (03:452-453)
# ----------------------------------------------------------------------------------------------


def mlp_fwd(x: torch.Tensor, layers: Sequence[Tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
    for w, b in layers:
        x = torch.relu(F.linear(x, w, b))
    return x


def dot_bce(q: torch.Tensor, c: torch.Tensor, labels: torch.Tensor):
    """logits = (q * c).sum(1).squeeze(); loss = BCEWithLogitsLoss()(logits, labels.float())."""
    logits = (q * c).sum(dim=1).squeeze()
    loss = nn.BCEWithLogitsLoss()(logits, labels.float())
    return logits, loss


def adam(params: List[torch.Tensor], grads: List[torch.Tensor], exp_avg, exp_avg_sq, step: int,
         lr: float, beta1=0.9, beta2=0.999, eps=1e-8) -> None:
    """torch.optim.Adam (amsgrad=False, weight_decay=0), single-tensor formula, in place."""
    for p, g, m, v in zip(params, grads, exp_avg, exp_avg_sq):
        m.lerp_(g, 1 - beta1)
        v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        bc1 = 1 - beta1 ** step
        bc2 = 1 - beta2 ** step
        denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
        p.addcdiv_(m, denom, value=-lr / bc1)


# ----------------------------------------------------------------------------------------------
# The whole training step on the CPU (TorchRec unsharded CPU semantics + fp32 towers)
# ----------------------------------------------------------------------------------------------


@dataclass
class TwoTowerState:
    """Parameters of the two-tower model: tables (one per feature key order given by
    feature_table), row-wise Adagrad state, and per-tower MLP layers [(W, b), ...]."""
    tables: List[torch.Tensor]
    states: List[torch.Tensor]
    feature_table: List[int]
    query_features: List[int]
    cand_features: List[int]
    dims: List[int]
    query_layers: List[Tuple[torch.Tensor, torch.Tensor]]
    cand_layers: List[Tuple[torch.Tensor, torch.Tensor]]
    exp_avg: List[torch.Tensor] = field(default_factory=list)
    exp_avg_sq: List[torch.Tensor] = field(default_factory=list)
    step: int = 0

    def dense_params(self) -> List[torch.Tensor]:
        return [t for wb in self.query_layers + self.cand_layers for t in wb]

    def clone(self) -> "TwoTowerState":
        c = lambda ts: [t.detach().clone() for t in ts]  # noqa: E731
        return TwoTowerState(
            c(self.tables), c(self.states), list(self.feature_table), list(self.query_features),
            list(self.cand_features), list(self.dims),
            [(w.detach().clone(), b.detach().clone()) for w, b in self.query_layers],
            [(w.detach().clone(), b.detach().clone()) for w, b in self.cand_layers],
            c(self.exp_avg), c(self.exp_avg_sq), self.step)


def feature_columns(dims: Sequence[int], features: Sequence[int]) -> List[int]:
    cols, off = [], 0
    starts = []
    for d in dims:
        starts.append(off)
        off += d
    for f in features:
        cols.extend(range(starts[f], starts[f] + dims[f]))
    return cols


def train_step(st: TwoTowerState, values: torch.Tensor, offsets: torch.Tensor, B: int,
               labels: torch.Tensor, lr_emb: float, lr_dense: float, eps: float = 1e-10,
               pooling: str = "sum", sparse_update: bool = True):
    """One step of 03_model_training.py's loop body (TrainPipelineSparseDist.progress): EBC
    forward, towers, dot + BCE (03:447-455), backward, fused RowWiseAdagrad on the tables
    (03:791-795) and Adam on the MLPs (03:826-829). Mutates st; returns (loss, logits, pooled,
    pooled_grad)."""
    pooled = pooled_fwd(st.tables, st.feature_table, values, offsets, B, pooling)
    pooled = pooled.detach().requires_grad_(True)
    dense = [p.detach().requires_grad_(True) for p in st.dense_params()]
    nq = len(st.query_layers)
    ql = [(dense[2 * i], dense[2 * i + 1]) for i in range(nq)]
    cl = [(dense[2 * nq + 2 * i], dense[2 * nq + 2 * i + 1]) for i in range(len(st.cand_layers))]
    qcols = feature_columns(st.dims, st.query_features)
    ccols = feature_columns(st.dims, st.cand_features)
    q = mlp_fwd(pooled[:, qcols], ql)
    c = mlp_fwd(pooled[:, ccols], cl)
    logits, loss = dot_bce(q, c, labels)
    loss.backward()
    gpooled = pooled.grad.detach()
    # embedding tables: dedup'd row gradients + row-wise Adagrad
    offs64 = offsets.to(torch.int64)
    for t in range(len(st.tables)):
        feats = [f for f, tt in enumerate(st.feature_table) if tt == t]
        if not feats:
            continue
        idxs, gs = [], []
        for f in feats:
            s, e = int(offs64[f * B]), int(offs64[(f + 1) * B])
            if e == s:
                continue
            idx = values[s:e].to(torch.int64)
            lens = (offs64[f * B + 1:(f + 1) * B + 1] - offs64[f * B:(f + 1) * B])
            bag = torch.repeat_interleave(torch.arange(B), lens)
            start = sum(st.dims[:f])
            g = gpooled[bag, start:start + st.dims[f]]
            if pooling == "mean":
                g = g / lens[bag].clamp(min=1).unsqueeze(1).to(g.dtype)
            idxs.append(idx)
            gs.append(g)
        if sparse_update:
            # compact [U, D] gradient of the touched rows only (same sums as the dense index_add)
            if not idxs:
                continue
            idx = torch.cat(idxs)
            rows, inv = torch.unique(idx, return_inverse=True)
            grad_rows = torch.zeros(rows.numel(), st.tables[t].shape[1])
            grad_rows.index_add_(0, inv, torch.cat(gs))
            rowwise_adagrad_sparse(st.tables[t], st.states[t], rows, grad_rows, lr_emb, eps)
        else:
            grad = torch.zeros_like(st.tables[t])
            for idx, g in zip(idxs, gs):
                grad.index_add_(0, idx, g)
            rowwise_adagrad(st.tables[t], st.states[t], grad, lr_emb, eps)
    # dense: Adam
    if not st.exp_avg:
        st.exp_avg = [torch.zeros_like(p) for p in st.dense_params()]
        st.exp_avg_sq = [torch.zeros_like(p) for p in st.dense_params()]
    st.step += 1
    params = st.dense_params()
    adam(params, [d.grad for d in dense], st.exp_avg, st.exp_avg_sq, st.step, lr_dense)
    return loss.detach(), logits.detach(), pooled.detach(), gpooled


def init_state(num_embeddings: Sequence[int], dims: Sequence[int], feature_table: Sequence[int],
               query_features: Sequence[int], cand_features: Sequence[int],
               layer_sizes: Sequence[int], seed: int = 0) -> TwoTowerState:
    """Deterministic initial parameters (CPU): tables U(-sqrt(1/N), sqrt(1/N)) (torchrec EBC
    default init), MLP nn.Linear default init."""
    g = torch.Generator().manual_seed(seed)
    tables = []
    for n, d in zip(num_embeddings, [dims[feature_table.index(t)] for t in range(len(num_embeddings))]):
        a = (1.0 / n) ** 0.5
        tables.append(torch.empty(n, d).uniform_(-a, a, generator=g))
    states = [torch.zeros(n) for n in num_embeddings]

    def mlp(in_size):
        layers = []
        for out in layer_sizes:
            bound = 1.0 / in_size ** 0.5
            w = torch.empty(out, in_size).uniform_(-bound, bound, generator=g)
            b = torch.empty(out).uniform_(-bound, bound, generator=g)
            layers.append((w, b))
            in_size = out
        return layers

    qin = sum(dims[f] for f in query_features)
    cin = sum(dims[f] for f in cand_features)
    return TwoTowerState(tables, states, list(feature_table), list(query_features), list(cand_features),
                         list(dims), mlp(qin), mlp(cin))


# ----------------------------------------------------------------------------------------------
# a10 (single-hot): sharded lookups — DistributedModelParallel + ShardedEmbeddingBagCollection
# (03_model_training.py:798-815): torchrec block_bucketize_sparse_features row-wise semantics
# (owner = row // ceil(N / W), local row = row - owner * block; EXTERNAL fbgemm-gpu 0.7.0
# sparse_ops block_bucketize, restated) or table-wise (whole table on one rank), with the
# fixed-capacity id exchange of csrc/shard.hip.
# ----------------------------------------------------------------------------------------------


def shard_route(cols: Sequence[np.ndarray], num_embeddings: Sequence[int], block_sizes: Sequence[int],
                owners: Sequence[int], W: int, C: int):
    """Returns (send [W, F + F*C] int64 — counts then keys f << 40 | local row, unused slots 0 —,
    pos [F*B] int32, overflow bool). Slot k of segment (d, f) = k-th kept lookup of feature f owned
    by d in ascending bag order (transform_to_torchrec_batch: id 0 dropped, id % N, 03:356-365)."""
    F = len(cols)
    B = len(cols[0])
    send = np.zeros((W, F + F * C), dtype=np.int64)
    pos = np.full(F * B, -1, dtype=np.int32)
    overflow = False
    for f in range(F):
        ids = np.asarray(cols[f]).astype(np.int64)
        cnt = np.zeros(W, dtype=np.int64)
        for b in range(B):
            if ids[b] == 0:
                continue
            row = int(np.mod(ids[b], num_embeddings[f]))
            if block_sizes[f] > 0:
                d, lr = row // block_sizes[f], row - (row // block_sizes[f]) * block_sizes[f]
            else:
                d, lr = owners[f], row
            k = cnt[d]
            cnt[d] += 1
            if k < C:
                send[d, F + f * C + k] = (f << 40) | lr
                pos[f * B + b] = (d * F + f) * C + k
            else:
                overflow = True
        for d in range(W):
            send[d, f] = min(cnt[d], C)
    return send, pos, overflow


def rowwise_adagrad_from_lookups(table: torch.Tensor, state: torch.Tensor, rows: torch.Tensor,
                                 grad_rows: torch.Tensor, lr: float, eps: float = 1e-10) -> None:
    """Fused backward of single-hot lookups: lookup j (row rows[j]) contributes grad_rows[j]; a
    row's lookups are summed in index order (dense index_add), then RowWiseAdagrad (03:791-795)."""
    if rows.numel() == 0:
        return
    u, inv = torch.unique(rows, return_inverse=True)
    g = torch.zeros(u.numel(), table.shape[1])
    g.index_add_(0, inv, grad_rows)
    rowwise_adagrad_sparse(table, state, u, g, lr, eps)


# ----------------------------------------------------------------------------------------------
# 8(f) row 3: evaluate() of 03_model_training.py:504-566 — forward only; AUROC of sigmoid(logits)
# over all batches (torchmetrics binary AUROC = scikit-learn roc_auc_score); average loss = the SUM
# of per-batch mean losses divided by the number of samples (the reference's quirk, 03:550-559)
# ----------------------------------------------------------------------------------------------


def evaluate(st: TwoTowerState, batches, num_embeddings: Sequence[int], limit_batches: Optional[int] = None):
    """batches: [(user ids, item ids, labels) numpy]; returns (avg_loss, auroc)."""
    from sklearn.metrics import roc_auc_score

    total, n, ps, ys = 0.0, 0, [], []
    for i, (u, it, lab) in enumerate(batches):
        if limit_batches is not None and i >= limit_batches:
            break
        v, _, o = kjt_build([u, it], num_embeddings)
        B = len(lab)
        pooled = pooled_fwd(st.tables, st.feature_table, torch.from_numpy(v).to(torch.int64), torch.from_numpy(o), B)
        q = mlp_fwd(pooled[:, feature_columns(st.dims, st.query_features)], st.query_layers)
        c = mlp_fwd(pooled[:, feature_columns(st.dims, st.cand_features)], st.cand_layers)
        logits, loss = dot_bce(q, c, torch.from_numpy(np.asarray(lab)))
        total += float(loss)
        n += B
        ps.append(torch.sigmoid(logits).numpy())
        ys.append(np.asarray(lab))
    return (total / n if n else 0.0), float(roc_auc_score(np.concatenate(ys), np.concatenate(ps)))
