import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box, `-m gpu`)")


def load_golden(name: str) -> dict:
    with np.load(GOLDEN / name, allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    # sparse_final fixtures (make_golden.py): dense final tables = initial tables with the changed
    # rows replaced; Adagrad states are zero outside them
    for k in [k for k in d if k.startswith("final_rows_")]:
        t = k[len("final_rows_"):]
        rows = d.pop(k)
        fin = d[f"init_{t}"].copy()
        fin[rows] = d.pop(f"final_vals_{t}")
        st = np.zeros(fin.shape[0], np.float32)
        st[rows] = d.pop(f"final_state_vals_{t}")
        d[f"final_{t}"], d[f"final_state_{t}"] = fin, st
    return d


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _release_gpu_memory(request):
    """After every GPU test: drop the caching allocator's free blocks, so tests that start child
    processes (each needs tens of GB of tables) never meet memory an earlier test left cached."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import gc

    import torch

    gc.collect()
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
