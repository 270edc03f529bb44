"""Deterministic CPU provider family ``stub-*`` (BASELINE config 1).

The reference has no CLI-selectable fake (``knownModels`` is closed, ``main.go:418-426``); this
family makes the whole CLI testable without a GPU and doubles as the fault-injection hook:

* ``stub-fail*``        → error ``stub: scripted failure`` before any token
* ``stub-slow*``        → blocks until its context ends (exercises ``--timeout``)
* ``stub-echo*``        → streams the prompt back
* ``stub-failat<k>*``   → streams k tokens then errors
* anything else         → a seeded pseudo-random token stream (synthetic tokenizer pieces)

``LLMC_STUB_TOKEN_MS`` adds a per-token delay so UI/progress paths can be observed.
"""

from __future__ import annotations

import os
import random
import re
import time
import zlib
from typing import Optional

from ..context import Context, ContextError
from ..utils.tokenizer import get_tokenizer
from .base import Request, Response, StreamCallback

STUB_VOCAB = 32000
DEFAULT_STUB_TOKENS = 24


class StubError(Exception):
    pass


class StubProvider:
    provider_name = "stub"

    def __init__(self, model: str, token_delay_s: Optional[float] = None):
        self.model = model
        if token_delay_s is None:
            token_delay_s = float(os.environ.get("LLMC_STUB_TOKEN_MS", "0")) / 1000.0
        self.token_delay_s = token_delay_s
        self.tok = get_tokenizer(STUB_VOCAB)

    def query(self, ctx: Context, req: Request) -> Response:
        return self.query_stream(ctx, req, None)

    def query_stream(self, ctx: Context, req: Request, callback: Optional[StreamCallback]) -> Response:
        t0 = time.monotonic_ns()
        family = req.model.partition("@")[0]
        if family.startswith("stub-fail") and not family.startswith("stub-failat"):
            raise StubError("stub: scripted failure")
        if family.startswith("stub-slow"):
            ctx.wait()
            raise ContextError(ctx.err())
        fail_at = None
        m = re.match(r"stub-failat(\d+)", family)
        if m:
            fail_at = int(m.group(1))
        if family.startswith("stub-echo"):
            ids = self.tok.encode(req.prompt)
        else:
            n = req.max_tokens if req.max_tokens else DEFAULT_STUB_TOKENS
            seed = zlib.crc32((req.model + "\x00" + req.prompt).encode("utf-8", "surrogatepass"))
            if req.seed is not None:
                seed ^= int(req.seed) & 0xFFFFFFFF
            rng = random.Random(seed)
            lo, hi = 256, 256 + self.tok._t.num_pieces - 1
            ids = [rng.randint(lo, hi) for _ in range(n)]
        dec = self.tok.stream_decoder()
        parts = []
        ttft = 0
        for i, t in enumerate(ids):
            ctx.check()
            if fail_at is not None and i == fail_at:
                raise StubError(f"stub: scripted failure at token {i}")
            if self.token_delay_s:
                time.sleep(self.token_delay_s)
            chunk = dec.push([t])
            if i == 0:
                ttft = time.monotonic_ns() - t0
            if chunk:
                parts.append(chunk)
                if callback is not None:
                    callback(chunk)
        tail = dec.flush()
        if tail:
            parts.append(tail)
            if callback is not None:
                callback(tail)
        return Response(model=req.model, content="".join(parts), provider=self.provider_name,
                        latency_ns=time.monotonic_ns() - t0, prompt_tokens=len(self.tok.encode(req.prompt)),
                        output_tokens=len(ids), ttft_ns=ttft)
