"""torchrec.distributed subset used by the reference (03_model_training.py:330-351)."""
from .model_parallel import DistributedModelParallel, get_default_sharders  # noqa: F401
from .train_pipeline import TrainPipelineBase, TrainPipelineSparseDist  # noqa: F401
from .types import ParameterSharding, ShardingPlan, ShardingType  # noqa: F401
