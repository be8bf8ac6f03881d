"""MI355X-native mirror of the torchrec API surface the reference's training loop uses
(03_model_training.py:330-351). Import it as ``torchrec`` with
``two_tower_recommender_model_amd.install_torchrec_alias()``."""
from .datasets.utils import Batch  # noqa: F401
from .modules.embedding_configs import EmbeddingBagConfig, PoolingType  # noqa: F401
from .modules.embedding_modules import EmbeddingBagCollection  # noqa: F401
from .modules.mlp import MLP  # noqa: F401
from .sparse.jagged_tensor import JaggedTensor, KeyedJaggedTensor, KeyedTensor  # noqa: F401
