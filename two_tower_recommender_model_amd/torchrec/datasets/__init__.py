from .utils import Batch  # noqa: F401
