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
