"""Host-side pieces of bench.py (no GPU): the multi-hot KJT synthesiser and the PMC-summary lookup."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_synth_kjt_batches_shapes_and_ranges():
    B, maxlen = 64, 7
    for ids in ("uniform", "zipf"):
        batches = bench.synth_kjt_batches(300, 500, B, maxlen, 2, torch.device("cpu"), ids, seed=1)
        for values, offsets, labels in batches:
            assert offsets.dtype == torch.int32 and offsets.numel() == 2 * B + 1 and int(offsets[0]) == 0
            lengths = offsets[1:] - offsets[:-1]
            assert int(lengths.min()) >= 1 and int(lengths.max()) <= maxlen
            assert values.numel() == int(offsets[-1])
            nb = int(offsets[B])
            assert int(values[:nb].max()) < 300 and int(values[nb:].max()) < 500 and int(values.min()) >= 0
            assert labels.numel() == B and set(labels.unique().tolist()) <= {0, 1}


def test_pmc_traffic_uses_the_benchmarked_workload():
    t, src = bench.pmc_traffic("tower_l2_kernel")
    assert src is None or ("config5" not in src and "zipf" not in src)
    t5, src5 = bench.pmc_traffic("bwd_adagrad_direct_kernel", "config5")
    assert src5 is None or "config5" in src5
    assert bench.pmc_traffic("tower_l2_kernel", "northstar_zipf") == (None, None)
