"""A small cancellation/deadline context modelled on Go's ``context.Context``.

The reference threads a ``context.Context`` through every query: the root is cancelled by
SIGINT/SIGTERM (``main.go:90``), each model gets ``context.WithTimeout`` (``runner.go:65``).
Engines check ``ctx.done()`` between decode steps, so cancellation latency is
one decode step (a few ms), not an HTTP abort.
"""

from __future__ import annotations

import threading
import time
from typing import List, Optional

DEADLINE_EXCEEDED = "context deadline exceeded"
CANCELED = "context canceled"


class ContextError(Exception):
    """Raised by providers when their context ends (message matches Go's ``ctx.Err()``)."""


class Context:
    def __init__(self, parent: Optional["Context"] = None, deadline: Optional[float] = None):
        self._parent = parent
        self._deadline = deadline
        if parent is not None and parent._deadline is not None:
            if self._deadline is None or parent._deadline < self._deadline:
                self._deadline = parent._deadline
        self._event = threading.Event()
        self._err: Optional[str] = None
        self._children: List["Context"] = []
        self._lock = threading.Lock()
        if parent is not None:
            with parent._lock:
                parent._children.append(self)
            if parent._err is not None:
                self._cancel(parent._err)

    # -- construction helpers -------------------------------------------------------------
    @staticmethod
    def background() -> "Context":
        return Context()

    def with_timeout(self, seconds: float) -> "Context":
        return Context(self, time.monotonic() + seconds)

    def with_cancel(self) -> "Context":
        return Context(self)

    # -- state ------------------------------------------------------------------------------
    @property
    def deadline(self) -> Optional[float]:
        return self._deadline

    def _cancel(self, err: str) -> None:
        with self._lock:
            if self._err is not None:
                return
            self._err = err
            children = list(self._children)
        self._event.set()
        for c in children:
            c._cancel(err)

    def cancel(self) -> None:
        self._cancel(CANCELED)

    def err(self) -> Optional[str]:
        if self._err is None and self._deadline is not None and time.monotonic() >= self._deadline:
            self._cancel(DEADLINE_EXCEEDED)
        return self._err

    def done(self) -> bool:
        return self.err() is not None

    def remaining(self) -> Optional[float]:
        if self._deadline is None:
            return None
        return max(0.0, self._deadline - time.monotonic())

    def wait(self, timeout: Optional[float] = None) -> bool:
        """Block until done or ``timeout``; returns ``done()``."""
        rem = self.remaining()
        if rem is not None:
            timeout = rem if timeout is None else min(timeout, rem)
        self._event.wait(timeout)
        return self.done()

    def check(self) -> None:
        e = self.err()
        if e is not None:
            raise ContextError(e)
