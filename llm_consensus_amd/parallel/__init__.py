from .comm import TPGroup, shard_range  # noqa: F401
