"""CPU: binary AUROC (metrics.py, the torchmetrics.AUROC(task="binary") the reference's evaluate()
uses, 03_model_training.py:524-551) against scikit-learn's roc_auc_score, ties included; the
torchmetrics alias."""
import numpy as np
import pytest
import torch
from sklearn.metrics import roc_auc_score

from two_tower_recommender_model_amd.metrics import AUROC, binary_auroc, install_torchmetrics_alias


@pytest.mark.parametrize("n,ties", [(10, False), (1000, False), (5000, True), (37, True)])
def test_binary_auroc_matches_sklearn(n, ties):
    rng = np.random.default_rng(n)
    y = rng.integers(0, 2, n)
    y[0], y[1] = 0, 1
    s = rng.normal(size=n) + 0.7 * y
    if ties:
        s = np.round(s, 1)
    got = float(binary_auroc(torch.from_numpy(s).float(), torch.from_numpy(y)))
    assert got == pytest.approx(roc_auc_score(y, s.astype(np.float32)), abs=1e-12)


def test_auroc_accumulates_batches_and_alias():
    rng = np.random.default_rng(0)
    m = AUROC(task="binary").to("cpu")
    ys, ss = [], []
    for _ in range(5):
        y = rng.integers(0, 2, 300)
        s = rng.random(300)
        m(torch.from_numpy(s), torch.from_numpy(y))
        ys.append(y)
        ss.append(s)
    assert float(m.compute()) == pytest.approx(roc_auc_score(np.concatenate(ys), np.concatenate(ss)), abs=1e-6)
    install_torchmetrics_alias()
    import torchmetrics

    assert hasattr(torchmetrics, "AUROC")
    assert torch.isnan(binary_auroc(torch.rand(4), torch.ones(4)))
