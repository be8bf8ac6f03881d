"""Generate the committed golden vectors by EXECUTING the reference's own hot-path code.

Run in the build container only (it reads /root/reference, which does not exist on the GPU box):

    python tests/golden/make_golden.py

What it does: parses /root/reference/03_model_training.py with ``ast`` and executes, unmodified,
the top-level definitions ``transform_to_torchrec_batch`` (03:353-380), ``TwoTower`` (03:395-437),
``TwoTowerTrainTask`` (03:440-455) and ``batched`` (03:467-470) in a namespace whose torchrec names
are bound to the CPU restatement in ``oracle/torchrec_cpu.py`` (torchrec itself is not installable
offline). The training step around them follows ``TrainPipelineSparseDist.progress``: forward,
``loss.backward()``, RowWiseAdagrad on the EBC tables (the in-backward optimizer of 03:791-795,
restated in oracle/ref.py) and ``torch.optim.Adam`` on the MLPs (KeyedOptimizerWrapper, 03:826-829).
Nothing from the reference is written out except these numeric inputs/outputs (npz fixtures).
"""
from __future__ import annotations

import ast
import itertools
import sys
from pathlib import Path
from typing import List, Optional, Tuple

import numpy as np
import torch
from torch import nn

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from oracle import ref  # noqa: E402
from oracle import torchrec_cpu as trc  # noqa: E402

REF_FILE = Path("/root/reference/03_model_training.py")
OUT = Path(__file__).resolve().parent
WANT = ("transform_to_torchrec_batch", "TwoTower", "TwoTowerTrainTask", "batched")


def load_reference_fragments(cat_cols):
    tree = ast.parse(REF_FILE.read_text())
    nodes = [n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name in WANT]
    assert sorted(n.name for n in nodes) == sorted(WANT), [n.name for n in nodes]
    mod = ast.Module(body=nodes, type_ignores=[])
    ns = dict(
        torch=torch, nn=nn, List=List, Optional=Optional, Tuple=Tuple, itertools=itertools,
        KeyedJaggedTensor=trc.KeyedJaggedTensor, Batch=trc.Batch,
        EmbeddingBagCollection=trc.EmbeddingBagCollection, MLP=trc.MLP, cat_cols=cat_cols,
    )
    exec(compile(mod, str(REF_FILE), "exec"), ns)
    return ns


def kjt_cases():
    """a1 golden vectors: the reference transform on int32/int64 columns with zeros, ids >= N,
    negative ids, and an all-zero batch."""
    cat_cols = ["user_id", "product_id"]
    ns = load_reference_fragments(cat_cols)
    g = torch.Generator().manual_seed(11)
    cases = {}
    specs = [
        ("i32", torch.int32, 64, [1000, 1500], 0.1),
        ("i64", torch.int64, 48, [777, 5], 0.2),
        ("big", torch.int64, 32, [3, 2**33 + 7], 0.0),
        ("allzero", torch.int32, 16, [10, 10], 1.0),
    ]
    for name, dt, B, N, pz in specs:
        cols = {}
        for ci, c in enumerate(cat_cols):
            hi = N[ci] * 3 if name != "big" else 2**40
            x = torch.randint(-N[ci], hi, (B,), generator=g, dtype=torch.int64)
            x[torch.rand(B, generator=g) < pz] = 0
            cols[c] = x.to(dt)
        cols["label"] = torch.randint(0, 2, (B,), generator=g, dtype=torch.int64)
        batch = ns["transform_to_torchrec_batch"](cols, num_embeddings_per_feature=N)
        kjt = batch.sparse_features
        cases[name] = dict(
            user_id=cols["user_id"].numpy(), product_id=cols["product_id"].numpy(), label=cols["label"].numpy(),
            num_embeddings=np.asarray(N, np.int64),
            values=kjt.values().numpy(), lengths=kjt.lengths().numpy(), offsets=kjt.offsets().numpy(),
            labels_out=batch.labels.numpy(),
        )
    for name, d in cases.items():
        np.savez_compressed(OUT / f"kjt_{name}.npz", **d)
    print("kjt cases:", list(cases))


def train_case(name, num_users, num_items, D, B, layers, steps, seed, zipf=False, lr=0.01, survey_ids=False,
               sparse_final=False):
    """a4-a9 golden vectors: ``steps`` training steps of the reference TwoTowerTrainTask.

    ``survey_ids``: SURVEY.md 8(d) config-1 ids (uniform in [1, N) plus 2 % zeros) instead of ids in
    [0, 2N) with 5 % zeros. ``sparse_final``: store the final tables / Adagrad states as the rows that
    differ from the initial ones (``final_rows_*`` / ``final_vals_*`` / ``final_state_vals_*``) to
    keep full-size fixtures small; tests/conftest.py:load_golden rebuilds the dense arrays."""
    cat_cols = ["user_id", "product_id"]
    ns = load_reference_fragments(cat_cols)
    torch.manual_seed(seed)
    g = torch.Generator().manual_seed(seed)
    emb_counts = [num_users, num_items]
    eb_configs = [
        trc.EmbeddingBagConfig(name=f"t_{f}", embedding_dim=D, num_embeddings=emb_counts[i], feature_names=[f])
        for i, f in enumerate(cat_cols)
    ]
    ebc = trc.EmbeddingBagCollection(tables=eb_configs)
    with torch.no_grad():  # torchrec EBC default init U(-sqrt(1/N), sqrt(1/N))
        for cfg in eb_configs:
            a = (1.0 / cfg.num_embeddings) ** 0.5
            ebc.embedding_bags[cfg.name].weight.uniform_(-a, a, generator=g)
    two_tower = ns["TwoTower"](embedding_bag_collection=ebc, layer_sizes=layers, device=None)
    task = ns["TwoTowerTrainTask"](two_tower)
    dense = [p for n, p in task.named_parameters() if "embedding_bags" not in n]
    adam = torch.optim.Adam(dense, lr=lr)
    states = [torch.zeros(n) for n in emb_counts]
    rec = {
        "init_t_user_id": ebc.embedding_bags["t_user_id"].weight.detach().clone().numpy(),
        "init_t_product_id": ebc.embedding_bags["t_product_id"].weight.detach().clone().numpy(),
        "layers": np.asarray(layers, np.int64), "D": np.int64(D), "B": np.int64(B), "steps": np.int64(steps),
        "num_embeddings": np.asarray(emb_counts, np.int64), "lr": np.float32(lr),
    }
    for n, p in task.named_parameters():
        if "embedding_bags" not in n:
            rec["init_" + n] = p.detach().clone().numpy()
    for s in range(steps):
        cols = {}
        for ci, c in enumerate(cat_cols):
            if zipf:
                r = torch.distributions.Pareto(1.0, 0.35).sample((B,)).floor().to(torch.int64)
                x = (r * 7919) % (emb_counts[ci] * 2)
            elif survey_ids:
                x = torch.randint(1, emb_counts[ci], (B,), generator=g, dtype=torch.int64)
            else:
                x = torch.randint(0, emb_counts[ci] * 2, (B,), generator=g, dtype=torch.int64)
            x[torch.rand(B, generator=g) < (0.02 if survey_ids else 0.05)] = 0
            cols[c] = x
        cols["label"] = torch.randint(0, 2, (B,), generator=g, dtype=torch.int64)
        batch = ns["transform_to_torchrec_batch"](cols, num_embeddings_per_feature=emb_counts)
        task.zero_grad(set_to_none=True)
        kt_holder = {}
        orig_fwd = ebc.forward

        def hooked(kjt):
            kt = orig_fwd(kjt)
            kt.values.retain_grad()
            kt_holder["kt"] = kt
            return kt

        ebc.forward = hooked
        loss, (loss_d, logits, labels) = task(batch)
        ebc.forward = orig_fwd
        loss.backward()
        pooled = kt_holder["kt"].values
        for ti, cfg in enumerate(eb_configs):
            wgt = ebc.embedding_bags[cfg.name].weight
            with torch.no_grad():
                ref.rowwise_adagrad(wgt.data, states[ti], wgt.grad, lr, 1e-10)
        adam.step()
        rec.update({
            f"s{s}_user_id": cols["user_id"].numpy(), f"s{s}_product_id": cols["product_id"].numpy(),
            f"s{s}_label": cols["label"].numpy(),
            f"s{s}_values": batch.sparse_features.values().numpy(),
            f"s{s}_offsets": batch.sparse_features.offsets().numpy(),
            f"s{s}_loss": loss_d.numpy(), f"s{s}_logits": logits.numpy(),
            f"s{s}_pooled": pooled.detach().numpy(), f"s{s}_pooled_grad": pooled.grad.numpy(),
        })
    for ti, cfg in enumerate(eb_configs):
        fin = ebc.embedding_bags[cfg.name].weight.detach().numpy()
        if sparse_final:
            rows = np.nonzero((fin != rec[f"init_{cfg.name}"]).any(1) | (states[ti].numpy() != 0))[0]
            rec[f"final_rows_{cfg.name}"] = rows.astype(np.int64)
            rec[f"final_vals_{cfg.name}"] = fin[rows]
            rec[f"final_state_vals_{cfg.name}"] = states[ti].numpy()[rows]
        else:
            rec[f"final_{cfg.name}"] = fin
            rec[f"final_state_{cfg.name}"] = states[ti].numpy()
    for n, p in task.named_parameters():
        if "embedding_bags" not in n:
            rec["final_" + n] = p.detach().numpy()
    np.savez_compressed(OUT / f"train_{name}.npz", **rec)
    print("train case:", name, "final loss", float(rec[f"s{steps-1}_loss"]))


class _SklearnAUROC:
    """Stand-in for torchmetrics.AUROC(task="binary") (not installable offline): exact binary AUROC
    of the accumulated scores via scikit-learn's roc_auc_score (same definition: trapezoidal ROC
    over distinct thresholds)."""

    def __init__(self, task="binary"):
        self.p, self.y = [], []

    def to(self, device):
        return self

    def __call__(self, preds, target):
        self.p.append(preds.detach().numpy().ravel())
        self.y.append(target.detach().numpy().ravel())

    def compute(self):
        from sklearn.metrics import roc_auc_score

        return torch.tensor(roc_auc_score(np.concatenate(self.y), np.concatenate(self.p)))


class _EvalPipeline:
    """What evaluate() touches of TrainPipelineSparseDist in eval mode: _model, _device, progress()."""

    def __init__(self, model):
        self._model = model
        self._device = torch.device("cpu")

    def progress(self, it):
        batch = next(it)
        with torch.no_grad():
            return self._model(batch)[1]


def eval_case(name, num_users, num_items, D, B, layers, n_batches, seed, limit_batches=None):
    """03:504-566 golden: the reference's own evaluate() (AST-extracted) on a fixed model state and
    fixed raw eval batches; records its (average loss, AUROC) return."""
    import functools
    import os
    import types

    import torch.distributed as dist

    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("gloo", rank=0, world_size=1)
    cat_cols = ["user_id", "product_id"]
    ns = load_reference_fragments(cat_cols)
    tree = ast.parse(REF_FILE.read_text())
    node = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "evaluate"][0]
    from tqdm import tqdm

    ns.update(dict(metrics=types.SimpleNamespace(AUROC=_SklearnAUROC), dist=dist, tqdm=tqdm,
                   TrainPipelineSparseDist=object, DataLoader=list, partial=functools.partial))
    exec(compile(ast.Module(body=[node], type_ignores=[]), str(REF_FILE), "exec"), ns)
    g = torch.Generator().manual_seed(seed)
    emb_counts = [num_users, num_items]
    eb_configs = [trc.EmbeddingBagConfig(name=f"t_{f}", embedding_dim=D, num_embeddings=emb_counts[i],
                                         feature_names=[f]) for i, f in enumerate(cat_cols)]
    ebc = trc.EmbeddingBagCollection(tables=eb_configs)
    with torch.no_grad():
        for cfg in eb_configs:
            ebc.embedding_bags[cfg.name].weight.uniform_(-0.3, 0.3, generator=g)
    torch.manual_seed(seed)
    task = ns["TwoTowerTrainTask"](ns["TwoTower"](embedding_bag_collection=ebc, layer_sizes=layers, device=None))
    task.eval()
    rec = {"D": np.int64(D), "B": np.int64(B), "layers": np.asarray(layers, np.int64),
           "num_embeddings": np.asarray(emb_counts, np.int64), "n_batches": np.int64(n_batches),
           "limit_batches": np.int64(-1 if limit_batches is None else limit_batches)}
    for n, p in task.named_parameters():
        rec["state_" + n] = p.detach().clone().numpy()
    raw = []
    for b in range(n_batches):
        cols = {c: torch.randint(0, 2 * emb_counts[i], (B,), generator=g, dtype=torch.int64)
                for i, c in enumerate(cat_cols)}
        cols["label"] = torch.randint(0, 2, (B,), generator=g, dtype=torch.int64)
        raw.append(cols)
        for k, v in cols.items():
            rec[f"b{b}_{k}"] = v.numpy()
    transform = functools.partial(ns["transform_to_torchrec_batch"], num_embeddings_per_feature=emb_counts)
    avg_loss, auroc = ns["evaluate"](limit_batches, _EvalPipeline(task), raw, "test", transform)
    rec["avg_loss"] = np.float64(avg_loss)
    rec["auroc"] = np.float64(auroc)
    np.savez_compressed(OUT / f"eval_{name}.npz", **rec)
    print("eval case:", name, avg_loss, auroc)


if __name__ == "__main__":
    import sys as _sys

    if len(_sys.argv) > 1 and _sys.argv[1] == "eval":
        eval_case("c1", num_users=700, num_items=900, D=32, B=256, layers=[32, 16], n_batches=5, seed=21)
        eval_case("limit", num_users=300, num_items=400, D=64, B=128, layers=[128, 64], n_batches=6, seed=22,
                  limit_batches=4)
        _sys.exit(0)
    if len(_sys.argv) > 1 and _sys.argv[1] == "c1full":
        train_case("c1full", num_users=10000, num_items=10000, D=16, B=256, layers=[128, 64], steps=3, seed=0,
                   survey_ids=True, sparse_final=True)
        _sys.exit(0)
    kjt_cases()
    # config-1 shape family (plumbing), shrunk to keep fixtures small
    train_case("c1", num_users=1000, num_items=1200, D=16, B=256, layers=[16, 8], steps=3, seed=0)
    train_case("zipf", num_users=500, num_items=800, D=32, B=128, layers=[32, 16], steps=3, seed=1, zipf=True)
    train_case("d128", num_users=300, num_items=400, D=128, B=64, layers=[128, 64], steps=2, seed=2)
    # config 1 at its full SURVEY.md 8(d) size: 10k x 10k, D=16, B=256, the reference's default
    # towers [128, 64] (03:62)
    train_case("c1full", num_users=10000, num_items=10000, D=16, B=256, layers=[128, 64], steps=3, seed=0,
               survey_ids=True, sparse_final=True)
