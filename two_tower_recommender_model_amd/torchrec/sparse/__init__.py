from .jagged_tensor import JaggedTensor, KeyedJaggedTensor, KeyedTensor  # noqa: F401
