"""torchrec.distributed subset used by the reference (03_model_training.py:330-351)."""
import os as _os

# the fused sharded drop-in captures RCCL collectives into HIP graphs: every ProcessGroupNCCL work
# needs its own event (sharded.graph_safe_nccl_env); the reference imports this package before its
# dist.init_process_group (03_model_training.py:751), which reads the variable
_os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")

from .model_parallel import DistributedModelParallel, get_default_sharders  # noqa: F401,E402
from .train_pipeline import TrainPipelineBase, TrainPipelineSparseDist  # noqa: F401,E402
from .types import ParameterSharding, ShardingPlan, ShardingType  # noqa: F401,E402
