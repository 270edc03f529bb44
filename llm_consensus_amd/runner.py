"""Best-effort N-model fan-out (reference ``internal/runner/runner.go:14-131``).

Semantics kept exactly:
* one concurrent task per entry of ``models`` (duplicates included, ``runner.go:62``);
* per-model deadline derived from the parent context (``runner.go:65``);
* ``on_model_start`` → registry lookup (failure = warning + failed, ``runner.go:73-83``) →
  streaming query forwarding chunks to ``on_model_stream``;
* results appended under a lock in COMPLETION order; ``on_model_error`` /
  ``on_model_complete`` fire while the lock is held (``runner.go:97-112``);
* error only when every model failed: ``all models failed: [w1 w2 ...]`` (``runner.go:122-124``);
  empty warnings / failed lists are ``None`` (Go nil slices, omitted by the JSON encoder).

On MI355X the "query" is a local engine generation; engines on different GPUs/streams run
truly in parallel because each provider call only enqueues work and waits on its own events —
threads here are I/O-style waiters, not compute.
"""

from __future__ import annotations

import dataclasses
import threading
from typing import Callable, List, Optional

from .context import Context
from .provider.base import Request, Response
from .provider.registry import Registry


@dataclasses.dataclass
class Callbacks:
    on_model_start: Optional[Callable[[str], None]] = None
    on_model_stream: Optional[Callable[[str, str], None]] = None
    # extension: exact generated-token counts from local engines (the UI shows them instead of
    # the reference's chars/4 estimate, ui.go:142)
    on_model_tokens: Optional[Callable[[str, int], None]] = None
    on_model_complete: Optional[Callable[[str], None]] = None
    on_model_error: Optional[Callable[[str, BaseException], None]] = None
    # Extension (no reference counterpart): the Response itself, called under the result lock
    # right after it is appended, i.e. in final slice order — drives incremental judge prefill.
    on_model_response: Optional[Callable[[Response], None]] = None


@dataclasses.dataclass
class RunResult:
    responses: List[Response]
    warnings: Optional[List[str]]
    failed_models: Optional[List[str]]


class AllModelsFailed(Exception):
    pass


def _fmt_list(items: List[str]) -> str:
    # Go's fmt "%v" of a []string: "[a b c]"
    return "[" + " ".join(items) + "]"


class Runner:
    def __init__(self, registry: Registry, timeout: float, request_template: Optional[Request] = None):
        self.registry = registry
        self.timeout = timeout
        self.callbacks: Optional[Callbacks] = None
        self._tmpl = request_template

    def with_callbacks(self, cb: Callbacks) -> "Runner":
        self.callbacks = cb
        return self

    def _request(self, model: str, prompt: str) -> Request:
        if self._tmpl is None:
            return Request(model=model, prompt=prompt)
        return dataclasses.replace(self._tmpl, model=model, prompt=prompt)

    def run(self, ctx: Context, models: List[str], prompt: str) -> RunResult:
        lock = threading.Lock()
        responses: List[Response] = []
        warnings: List[str] = []
        failed: List[str] = []
        cb = self.callbacks

        def task(model: str) -> None:
            mctx = ctx.with_timeout(self.timeout)
            if cb and cb.on_model_start:
                cb.on_model_start(model)
            try:
                p = self.registry.get(model)
            except Exception as e:  # noqa: BLE001
                with lock:
                    warnings.append(f"{model}: {e}")
                    failed.append(model)
                if cb and cb.on_model_error:
                    cb.on_model_error(model, e)
                return

            def stream(chunk: str) -> None:
                if cb and cb.on_model_stream:
                    cb.on_model_stream(model, chunk)

            if cb and cb.on_model_tokens:
                stream.tokens_hook = lambda n, _m=model: cb.on_model_tokens(_m, n)  # type: ignore[attr-defined]

            err: Optional[BaseException] = None
            resp: Optional[Response] = None
            try:
                resp = p.query_stream(mctx, self._request(model, prompt), stream)
            except Exception as e:  # noqa: BLE001 - best effort: any failure is per-model
                err = e
            with lock:
                if err is not None:
                    warnings.append(f"{model}: {err}")
                    failed.append(model)
                    if cb and cb.on_model_error:
                        cb.on_model_error(model, err)
                    return
                responses.append(resp)
                if cb and cb.on_model_response:
                    cb.on_model_response(resp)
                if cb and cb.on_model_complete:
                    cb.on_model_complete(model)

        threads = [threading.Thread(target=task, args=(m,), daemon=True, name=f"runner:{m}") for m in models]
        for t in threads:
            t.start()
        for t in threads:
            t.join()

        if not responses:
            raise AllModelsFailed("all models failed: " + _fmt_list(warnings))
        return RunResult(responses=responses, warnings=warnings or None, failed_models=failed or None)
