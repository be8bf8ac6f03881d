from .keyed import KeyedOptimizer, KeyedOptimizerWrapper  # noqa: F401
from .rowwise_adagrad import RowWiseAdagrad  # noqa: F401
