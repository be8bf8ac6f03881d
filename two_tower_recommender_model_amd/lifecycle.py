"""Checkpoint, evaluation and embedding export around the fused steps (SURVEY.md section 8(f) rows
2-4), in the reference's formats.

* Checkpoint (03_model_training.py:474-502 writes, :1015-1054 reads): the gathered state dict of
  ``TwoTowerTrainTask`` — keys ``two_tower.ebc.embedding_bags.t_<feature>.weight`` (full tables,
  fp32), ``two_tower.query_proj._mlp.<l>._linear.{weight,bias}`` and ``candidate_proj`` alike —
  which ``get_mlflow_model`` strips of "two_tower." (k[10:]) and loads into TwoTower. The optimizer
  state (row-wise Adagrad sums, Adam moments and step), absent from the reference, is a second dict
  so training can resume bit-exactly.
* Evaluation (03:504-566): forward only over a stream of batches; AUROC of sigmoid(logits)
  (torchmetrics binary AUROC, metrics.py) and the reference's average loss, which divides the SUM
  OF PER-BATCH MEAN LOSSES by the number of samples (03:550-559) — kept as is, with the per-sample
  mean reported beside it.
* Embedding export (03:1056-1122, :1160-1240): every row of a table through its tower (EBC of a
  one-id bag = the row itself, then the MLP with ReLU on every layer); row i is labelled id i + 1
  as the reference does (:1168, :1235), which is NOT the training map id -> id % N (03:361).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from . import ops
from .metrics import AUROC

DEFAULT_FEATURES = ("user_id", "product_id")  # cat_cols of 03_model_training.py:39


def _tower_views(params: torch.Tensor, in_dims: Sequence[int], layer_sizes: Sequence[int]):
    """[(W, b)] per tower from the flat parameter buffer (tt_tower_shape_t layout)."""
    out, o = [], 0
    for t in range(2):
        layers, i = [], in_dims[t]
        for n in layer_sizes:
            w = params[o:o + n * i].view(n, i)
            o += n * i
            b = params[o:o + n]
            o += n
            layers.append((w, b))
            i = n
        out.append(layers)
    return out


def _dense_items(towers, prefix: str):
    items = {}
    for name, layers in zip(("query_proj", "candidate_proj"), towers):
        for l, (w, b) in enumerate(layers):
            items[f"{prefix}{name}._mlp.{l}._linear.weight"] = w
            items[f"{prefix}{name}._mlp.{l}._linear.bias"] = b
    return items


# ---- single-GPU fused step ---------------------------------------------------------------------


def fused_state_dict(step, feature_names: Sequence[str] = DEFAULT_FEATURES,
                     prefix: str = "two_tower.") -> Dict[str, torch.Tensor]:
    """The reference's gathered state dict of the model trained by a FusedTwoTowerStep (one table
    per feature, feature f -> table t_<feature f>). Tensors are copies on the step's device."""
    sd = {}
    for f, name in enumerate(feature_names):
        sd[f"{prefix}ebc.embedding_bags.t_{name}.weight"] = step.tables.table_view(f).clone()
    towers = _tower_views(step.params, [step.in_q, step.in_c], step.layer_sizes)
    sd.update({k: v.clone() for k, v in _dense_items(towers, prefix).items()})
    return sd


def load_fused_state_dict(step, sd: Dict[str, torch.Tensor], feature_names: Sequence[str] = DEFAULT_FEATURES,
                          prefix: str = "two_tower.") -> None:
    """Inverse of fused_state_dict (a reference checkpoint loads as is); refreshes the towers' bf16
    weight copies."""
    with torch.no_grad():
        for f, name in enumerate(feature_names):
            step.tables.table_view(f).copy_(sd[f"{prefix}ebc.embedding_bags.t_{name}.weight"])
        towers = _tower_views(step.params, [step.in_q, step.in_c], step.layer_sizes)
        for k, v in _dense_items(towers, prefix).items():
            v.copy_(sd[k])
    step.sync_weights()


def fused_optimizer_state(step) -> Dict[str, torch.Tensor]:
    """Row-wise Adagrad sums of every table, Adam moments and step counter (resume state)."""
    st = {f"rowwise_adagrad.t{f}.momentum1": step.tables.state_view(f).clone() for f in range(step.F)}
    st.update({"adam.exp_avg": step.exp_avg.clone(), "adam.exp_avg_sq": step.exp_avg_sq.clone(),
               "adam.step": step.adam_state.clone()})
    return st


def load_fused_optimizer_state(step, st: Dict[str, torch.Tensor]) -> None:
    with torch.no_grad():
        for f in range(step.F):
            step.tables.state_view(f).copy_(st[f"rowwise_adagrad.t{f}.momentum1"])
        step.exp_avg.copy_(st["adam.exp_avg"])
        step.exp_avg_sq.copy_(st["adam.exp_avg_sq"])
        step.adam_state.copy_(st["adam.step"])


# ---- evaluation ----------------------------------------------------------------------------------


def evaluate_fused(step, batches: Iterable[Tuple[Sequence[torch.Tensor], torch.Tensor]],
                   limit_batches: Optional[int] = None) -> Dict[str, float]:
    """evaluate() of 03_model_training.py:504-566 on a FusedTwoTowerStep: forward only (no table or
    tower update), AUROC over all batches, and the reference's average loss (sum of batch means
    / samples). Returns {"avg_loss", "auroc", "mean_loss", "batches", "samples"}."""
    auroc = AUROC(task="binary").to(step.device)
    total_loss = torch.zeros((), dtype=torch.float64, device=step.device)
    n_batches = n_samples = 0
    for i, (cols, labels) in enumerate(batches):
        if limit_batches is not None and i >= limit_batches:
            break
        loss, logits = step.eval_step(cols, labels)
        auroc(torch.sigmoid(logits), labels)
        total_loss += loss.to(torch.float64)
        n_batches += 1
        n_samples += labels.numel()
    total = float(total_loss)
    return {"avg_loss": total / n_samples if n_samples else 0.0, "auroc": float(auroc.compute()),
            "mean_loss": total / n_batches if n_batches else 0.0, "batches": n_batches, "samples": n_samples}


# ---- embedding export ----------------------------------------------------------------------------


def export_embeddings(table: torch.Tensor, layers: Sequence[Tuple[torch.Tensor, torch.Tensor]],
                      chunk: int = 1 << 20, precision: str = "bf16",
                      out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """process_embeddings (03:1089-1117) for every row of ``table`` ([N, D] fp32, device): the
    tower MLP (Linear + ReLU on every layer) on bf16 MFMA GEMMs (fp32 accumulate; "fp32" for the
    exact path), ``chunk`` rows per launch. Returns (ids = arange(N) + 1 — the reference's labels —,
    embeddings [N, out])."""
    N = table.shape[0]
    width = layers[-1][0].shape[0]
    if out is None:
        out = torch.empty(N, width, dtype=torch.float32, device=table.device)
    for lo in range(0, N, chunk):
        x = table[lo:lo + chunk]
        for l, (w, b) in enumerate(layers):
            y = out[lo:lo + chunk] if l == len(layers) - 1 else None
            x = ops.linear_fwd([x], [w.contiguous()], [b], relu=True, outs=[y] if y is not None else None,
                               precision=precision)[0]
    ids = torch.arange(1, N + 1, dtype=torch.int64, device=table.device)
    return ids, out


def export_fused(step, tower: str = "candidate", **kw) -> Tuple[torch.Tensor, torch.Tensor]:
    """export_embeddings of a FusedTwoTowerStep's item ("candidate", table 1) or user ("query",
    table 0) tower."""
    t = 1 if tower == "candidate" else 0
    towers = _tower_views(step.params, [step.in_q, step.in_c], step.layer_sizes)
    return export_embeddings(step.tables.table_view(t), towers[t], **kw)
