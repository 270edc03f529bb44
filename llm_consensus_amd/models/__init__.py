from .config import FAMILIES, ModelConfig  # noqa: F401
