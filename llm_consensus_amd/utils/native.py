"""Loaders for the two in-tree native modules (see ``llm_consensus_amd/_build.py``).

``runtime()`` builds the host runtime on first use if it is missing (g++ only, seconds).
``kernels()`` loads the HIP kernel module and raises loudly if it is absent — CUDA tensors
never fall back to PyTorch ops (the round-end checker records which in-tree ``.so`` files
a GPU run actually loaded).
"""

from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_rt = None
_hip = None


def runtime():
    global _rt
    if _rt is not None:
        return _rt
    with _lock:
        if _rt is None:
            from .. import _build

            if not os.path.exists(_build.runtime_path()) or os.environ.get("LLMC_REBUILD"):
                _build.build_runtime()
            _rt = importlib.import_module("llm_consensus_amd._lib._llmc_rt")
    return _rt


def kernels():
    global _hip
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is None:
            from .. import _build

            path = _build.kernels_path()
            if not os.path.exists(path):
                if os.environ.get("LLMC_AUTOBUILD", "1") == "1":
                    _build.build_kernels()
                else:
                    raise RuntimeError(f"HIP kernel module missing: {path}; run `python -m llm_consensus_amd._build`")
            _hip = importlib.import_module("llm_consensus_amd._lib._llmc_hip")
    return _hip
