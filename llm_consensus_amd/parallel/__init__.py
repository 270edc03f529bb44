"""Parallel layer: placement (torch-free: the CLI driver plans placements without importing
torch), TP communication (``comm``) and the custom xGMI collectives (``custom_ar``). ``TPGroup``
and ``shard_range`` resolve lazily from ``comm``."""


def __getattr__(name):
    if name in ("TPGroup", "shard_range"):
        from . import comm

        return getattr(comm, name)
    raise AttributeError(name)
