"""DistributedModelParallel -> ShardedEmbeddingBagCollection with the HIP backend on the GPU, over a
one-rank RCCL group (tests/dmp_nccl_check.py): TW + RW shards, multi-hot bags, a shared table,
towers over concatenated features, training through TrainPipelineSparseDist and KeyedOptimizer-
Wrapper(Adam), then eval mode — against the oracle. Run in a child process."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_dmp_sharded_ebc_hip_backend_vs_oracle(device):
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "dmp_nccl_check.py")], capture_output=True, text=True,
                       timeout=300, cwd=os.path.dirname(here))
    assert r.returncode == 0 and "DMP-NCCL-OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])


def test_dmp_config3_shape_world1(device):
    """BASELINE config 3's shape (16 single-hot TW tables, 8 features per tower, 50M / 100M / 14 x 1M
    rows, D 128, B 8192, 1024-wide tower inputs) through DMP -> ShardedEBC (HIP) ->
    TrainPipelineSparseDist on one rank, against the oracle on the touched rows
    (tests/dmp_config3_check.py)."""
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "dmp_config3_check.py")], capture_output=True, text=True,
                       timeout=600, cwd=os.path.dirname(here))
    assert r.returncode == 0 and "DMP-CONFIG3-OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
