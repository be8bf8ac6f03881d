"""DistributedModelParallel -> ShardedEmbeddingBagCollection with the HIP backend on the GPU, over a
one-rank RCCL group (tests/dmp_nccl_check.py): TW + RW shards, multi-hot bags, a shared table,
towers over concatenated features, training through TrainPipelineSparseDist and KeyedOptimizer-
Wrapper(Adam), then eval mode — against the oracle. Run in a child process."""
import pytest

from child_util import run_child

pytestmark = pytest.mark.gpu


def test_dmp_sharded_ebc_hip_backend_vs_oracle(device):
    run_child(["tests/dmp_nccl_check.py"], "DMP-NCCL-OK", timeout=300)


def test_dmp_config3_shape_world1(device):
    """BASELINE config 3's shape (16 single-hot TW tables, 8 features per tower, 50M / 100M / 14 x 1M
    rows, D 128, B 8192, 1024-wide tower inputs) through DMP -> ShardedEBC (HIP) ->
    TrainPipelineSparseDist on one rank, against the oracle on the touched rows
    (tests/dmp_config3_check.py)."""
    run_child(["tests/dmp_config3_check.py"], "DMP-CONFIG3-OK", timeout=600)
