"""Provider API (reference ``internal/provider/provider.go:8-55``).

``Provider.query_stream(ctx, req, callback) -> Response`` is the single contract every model
backend implements: the callback receives incremental text chunks and the returned
``content`` is their concatenation; ``latency`` spans request start → end of stream
(``openai.go:142, 208``).  ``FuncProvider`` is the test fake (``provider.go:37-55``): it calls
the function and then invokes the callback once with the full content.

Deviation: the JSON field ``latency_ms`` carries milliseconds; the raw
nanosecond value is kept in ``latency_ns`` for benches.
"""

from __future__ import annotations

import dataclasses
from typing import Callable, Optional, Protocol

from ..context import Context

StreamCallback = Callable[[str], None]


@dataclasses.dataclass
class Request:
    model: str
    prompt: str
    # Engine knobs (no reference counterpart: the reference sends model+prompt only,
    # provider.go:24-27). ``None`` = engine default.
    max_tokens: Optional[int] = None
    temperature: Optional[float] = None
    top_p: Optional[float] = None
    top_k: Optional[int] = None
    seed: Optional[int] = None
    stop_on_eos: Optional[bool] = None  # None = stop at the model's EOS (benchmarks pin full lengths)


@dataclasses.dataclass
class Response:
    model: str = ""
    content: str = ""
    provider: str = ""
    latency_ns: int = 0
    # Non-schema statistics (not serialised into result.json).
    prompt_tokens: int = 0
    output_tokens: int = 0
    ttft_ns: int = 0

    @property
    def latency_ms(self) -> int:
        return self.latency_ns // 1_000_000

    @property
    def latency_s(self) -> float:
        return self.latency_ns / 1e9


class Provider(Protocol):
    def query(self, ctx: Context, req: Request) -> Response: ...

    def query_stream(self, ctx: Context, req: Request, callback: Optional[StreamCallback]) -> Response: ...


class FuncProvider:
    """Adapter turning ``fn(ctx, req) -> Response`` into a Provider (``provider.go:37-55``)."""

    def __init__(self, fn: Callable[[Context, Request], Response]):
        self._fn = fn

    def query(self, ctx: Context, req: Request) -> Response:
        return self._fn(ctx, req)

    def query_stream(self, ctx: Context, req: Request, callback: Optional[StreamCallback]) -> Response:
        resp = self._fn(ctx, req)
        if callback is not None:
            callback(resp.content)
        return resp
