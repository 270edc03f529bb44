from .engine import Engine, EngineConfig, EngineError, SamplingParams, Sequence  # noqa: F401
