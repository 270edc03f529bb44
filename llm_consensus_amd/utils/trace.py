"""Chrome-trace span recorder + roctx ranges.

``span("prefill", engine="llama-3-8b@0")`` records a complete event (ph="X") when tracing is
enabled (``--trace`` or ``LLMC_TRACE=1``) and, on a GPU process, also pushes a roctx range so
``rocprofv3 --marker-trace`` lines kernel activity up with engine phases. Worker processes send
their events to the driver, which writes ``data/<run-id>/trace.json``.
"""

from __future__ import annotations

import contextlib
import json
import os
import sys
import threading
import time
from typing import Dict, List

_enabled = os.environ.get("LLMC_TRACE", "0") == "1"
_lock = threading.Lock()
_events: List[Dict] = []
# Timestamps: CLOCK_MONOTONIC, which is system-wide on Linux, so the driver's and every worker's
# events share one time axis in the merged trace (a per-process origin would shift them apart).


def _now_us() -> float:
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC) / 1000.0


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = on


def enabled() -> bool:
    return _enabled


def _roctx():
    """roctx in processes that already run torch (the GPU workers); the torch-free driver never
    imports it for a trace span (a ~2 s import inside a query's span)."""
    torch = sys.modules.get("torch")
    if torch is None:
        return None
    try:
        if torch.cuda.is_available() and hasattr(torch.cuda, "nvtx"):
            return torch.cuda.nvtx
    except Exception:  # noqa: BLE001
        pass
    return None


@contextlib.contextmanager
def span(name: str, cat: str = "engine", **args):
    if not _enabled:
        yield
        return
    rx = _roctx()
    if rx is not None:
        try:
            rx.range_push(name)
        except Exception:  # noqa: BLE001
            rx = None
    t = _now_us()
    try:
        yield
    finally:
        d = _now_us() - t
        if rx is not None:
            rx.range_pop()
        ev = {"name": name, "cat": cat, "ph": "X", "ts": t, "dur": d,
              "pid": os.getpid(), "tid": threading.get_ident() % 100000, "args": args}
        with _lock:
            _events.append(ev)


def instant(name: str, cat: str = "engine", **args) -> None:
    if not _enabled:
        return
    ev = {"name": name, "cat": cat, "ph": "i", "s": "p", "ts": _now_us(),
          "pid": os.getpid(), "tid": threading.get_ident() % 100000, "args": args}
    with _lock:
        _events.append(ev)


def add_events(evs: List[Dict]) -> None:
    with _lock:
        _events.extend(evs)


def drain() -> List[Dict]:
    with _lock:
        out = list(_events)
        _events.clear()
    return out


def dump(path: str) -> None:
    with _lock:
        data = {"traceEvents": list(_events), "displayTimeUnit": "ms"}
    with open(path, "w") as f:
        json.dump(data, f)
