"""Remote API providers, kept so a reference user can still mix hosted models into a run.

The reference's only backends are these three HTTP adapters (``internal/provider/openai.go``,
``anthropic.go``, ``google.go``); here they sit beside the local MI355X engines behind the same
``query`` / ``query_stream`` contract (``provider.go:13-21``). Wire behaviour follows the
reference:

* OpenAI Responses API: ``POST {base}/responses`` with ``{"model", "input"[, "stream": true]}``,
  ``Authorization: Bearer $OPENAI_API_KEY``; streamed text = ``response.output_text.delta``
  events, ``[DONE]`` ends the stream; non-streamed text = every ``output_text`` part of every
  ``message`` output item, empty content is an error (openai.go:82-261).
* Anthropic Messages API: ``POST {base}/messages`` with ``max_tokens`` 4096 and one user message,
  headers ``x-api-key`` and ``anthropic-version: 2023-06-01``; streamed text =
  ``content_block_delta`` events whose delta is ``text_delta`` (anthropic.go:52-234).
* Google Gemini: ``POST {base}/models/{model}:generateContent?key=...`` /
  ``:streamGenerateContent?key=...&alt=sse``; text = ``candidates[0].content.parts[0].text``
  (google.go:53-230).
* SSE lines not starting with ``data: `` are skipped and undecodable JSON lines are ignored;
  a non-200 status is ``API error (status N): <body>``; the latency spans request start to the
  end of the stream.

Deliberate deviation: no hidden 60 s client cap — the run's per-model context
deadline (``--timeout``) bounds the request, and cancellation closes the stream. Base URLs can be
overridden (``OPENAI_BASE_URL`` / ``ANTHROPIC_BASE_URL`` / ``GOOGLE_BASE_URL``), the analogue of the
reference's ``With*BaseURL`` options, which the tests use to point at a local mock server.
"""

from __future__ import annotations

import json
import os
import time
from typing import Iterator, Optional

from ..context import Context, ContextError
from .base import Request, Response, StreamCallback

PROVIDER_OPENAI, PROVIDER_ANTHROPIC, PROVIDER_GOOGLE = "openai", "anthropic", "google"

# reference catalog: cmd/llm-consensus/main.go:47-61
KNOWN_REMOTE = {
    "gpt-5.2-2025-12-11": PROVIDER_OPENAI,
    "gpt-5.2-pro-2025-12-11": PROVIDER_OPENAI,
    "claude-sonnet-4-5": PROVIDER_ANTHROPIC,
    "claude-haiku-4-5": PROVIDER_ANTHROPIC,
    "claude-opus-4-5": PROVIDER_ANTHROPIC,
    "gemini-3-pro-preview": PROVIDER_GOOGLE,
}


class RemoteError(Exception):
    pass


def _client():
    import httpx

    return httpx.Client(timeout=httpx.Timeout(connect=30.0, read=None, write=30.0, pool=30.0))


def _remaining(ctx: Context) -> Optional[float]:
    r = ctx.remaining()
    return None if r is None else max(0.001, r)


class _HTTPProvider:
    provider_name = ""
    env_key = ""
    env_base = ""
    default_base = ""

    def __init__(self, model: str, api_key: Optional[str] = None, base_url: Optional[str] = None):
        key = api_key if api_key is not None else os.environ.get(self.env_key, "")
        if not key:
            raise RemoteError(f"{self.env_key} environment variable required")
        self.model = model
        self.api_key = key
        self.base_url = (base_url or os.environ.get(self.env_base) or self.default_base).rstrip("/")

    # -- subclass hooks ------------------------------------------------------------------------
    def _request(self, req: Request, stream: bool):  # -> (url, headers, body)
        raise NotImplementedError

    def _text_of(self, body: dict) -> str:
        raise NotImplementedError

    def _delta_of(self, event: dict) -> Optional[str]:
        raise NotImplementedError

    # -- shared plumbing -----------------------------------------------------------------------
    def _post(self, ctx: Context, req: Request, stream: bool):
        import httpx

        url, headers, body = self._request(req, stream)
        client = _client()
        try:
            r = client.send(client.build_request("POST", url, headers=headers, json=body,
                                                 timeout=httpx.Timeout(_remaining(ctx), connect=30.0)),
                            stream=True)
        except httpx.HTTPError as e:
            client.close()
            raise RemoteError(f"sending request: {e}") from None
        if r.status_code != 200:
            data = r.read().decode("utf-8", "replace")
            r.close()
            client.close()
            raise RemoteError(f"API error (status {r.status_code}): {data}")
        return client, r

    def query(self, ctx: Context, req: Request) -> Response:
        t0 = time.monotonic_ns()
        client, r = self._post(ctx, req, stream=False)
        try:
            raw = r.read()
        finally:
            r.close()
            client.close()
        try:
            body = json.loads(raw)
        except ValueError as e:
            raise RemoteError(f"parsing response: {e}") from None
        text = self._text_of(body)
        if not text:
            raise RemoteError("no content in response")
        return Response(model=req.model, content=text, provider=self.provider_name,
                        latency_ns=time.monotonic_ns() - t0)

    def query_stream(self, ctx: Context, req: Request, callback: Optional[StreamCallback]) -> Response:
        import httpx

        t0 = time.monotonic_ns()
        client, r = self._post(ctx, req, stream=True)
        parts = []
        ttft = 0
        try:
            for data in _sse_data(r.iter_lines(), ctx):
                if data == "[DONE]":
                    break
                try:
                    event = json.loads(data)
                except ValueError:
                    continue  # undecodable lines are skipped (openai.go:185-187)
                chunk = self._delta_of(event)
                if chunk:
                    if not ttft:
                        ttft = time.monotonic_ns() - t0
                    parts.append(chunk)
                    if callback is not None:
                        callback(chunk)
        except httpx.HTTPError as e:
            raise RemoteError(f"reading stream: {e}") from None
        finally:
            r.close()
            client.close()
        return Response(model=req.model, content="".join(parts), provider=self.provider_name,
                        latency_ns=time.monotonic_ns() - t0, ttft_ns=ttft)


def _sse_data(lines: Iterator[str], ctx: Context) -> Iterator[str]:
    for line in lines:
        if ctx.done():
            raise ContextError(ctx.err())
        if line.startswith("data: "):
            yield line[len("data: "):]


class OpenAIProvider(_HTTPProvider):
    provider_name = PROVIDER_OPENAI
    env_key = "OPENAI_API_KEY"
    env_base = "OPENAI_BASE_URL"
    default_base = "https://api.openai.com/v1"

    def _request(self, req, stream):
        body = {"model": req.model, "input": req.prompt}
        if stream:
            body["stream"] = True
        return (f"{self.base_url}/responses",
                {"Content-Type": "application/json", "Authorization": f"Bearer {self.api_key}"}, body)

    def _text_of(self, body):
        out = []
        for item in body.get("output") or []:
            if item.get("type") == "message":
                for c in item.get("content") or []:
                    if c.get("type") == "output_text":
                        out.append(c.get("text", ""))
        return "".join(out)

    def _delta_of(self, event):
        return event.get("delta") if event.get("type") == "response.output_text.delta" else None


class AnthropicProvider(_HTTPProvider):
    provider_name = PROVIDER_ANTHROPIC
    env_key = "ANTHROPIC_API_KEY"
    env_base = "ANTHROPIC_BASE_URL"
    default_base = "https://api.anthropic.com/v1"
    max_tokens = 4096  # anthropic.go:79, 137

    def _request(self, req, stream):
        body = {"model": req.model, "max_tokens": self.max_tokens,
                "messages": [{"role": "user", "content": req.prompt}]}
        if stream:
            body["stream"] = True
        return (f"{self.base_url}/messages",
                {"Content-Type": "application/json", "x-api-key": self.api_key, "anthropic-version": "2023-06-01"},
                body)

    def _text_of(self, body):
        return "".join(c.get("text", "") for c in body.get("content") or [] if c.get("type", "text") == "text")

    def _delta_of(self, event):
        d = event.get("delta") or {}
        if event.get("type") == "content_block_delta" and d.get("type") == "text_delta":
            return d.get("text")
        return None


class GoogleProvider(_HTTPProvider):
    provider_name = PROVIDER_GOOGLE
    env_key = "GOOGLE_API_KEY"
    env_base = "GOOGLE_BASE_URL"
    default_base = "https://generativelanguage.googleapis.com/v1beta"

    def _request(self, req, stream):
        body = {"contents": [{"parts": [{"text": req.prompt}]}]}
        verb = "streamGenerateContent" if stream else "generateContent"
        suffix = "&alt=sse" if stream else ""
        return (f"{self.base_url}/models/{req.model}:{verb}?key={self.api_key}{suffix}",
                {"Content-Type": "application/json"}, body)

    def _text_of(self, body):
        c = body.get("candidates") or []
        if not c or not ((c[0].get("content") or {}).get("parts")):
            return ""
        return c[0]["content"]["parts"][0].get("text", "")

    def _delta_of(self, event):
        return self._text_of(event) or None


FACTORIES: dict = {PROVIDER_OPENAI: OpenAIProvider, PROVIDER_ANTHROPIC: AnthropicProvider,
                   PROVIDER_GOOGLE: GoogleProvider}


def create(model: str, kind: str) -> _HTTPProvider:
    """createProvider (main.go:417-438) for a remote model."""
    return FACTORIES[kind](model)
