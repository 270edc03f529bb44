"""Remote API adapters (reference internal/provider/{openai,anthropic,google}.go) against a local
mock server speaking each API's wire format: requests (path, headers, body), streamed SSE
parsing (skipped non-data lines, undecodable JSON, [DONE]), non-streamed extraction, API errors,
and the CLI mixing hosted models with a stub judge."""

import json
import os
import subprocess
import sys
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from llm_consensus_amd.context import Context
from llm_consensus_amd.provider.base import Request
from llm_consensus_amd.provider.remote import (AnthropicProvider, GoogleProvider, OpenAIProvider, RemoteError,
                                               create)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEEN = []


class _H(BaseHTTPRequestHandler):
    def log_message(self, *a):
        pass

    def _sse(self, lines):
        self.send_response(200)
        self.send_header("Content-Type", "text/event-stream")
        self.end_headers()
        for ln in lines:
            self.wfile.write((ln + "\n").encode())
            self.wfile.flush()

    def _json(self, obj, code=200):
        data = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def do_GET(self):
        SEEN.append((self.path, dict(self.headers), None))
        if self.path == "/oa/models":
            return self._json({"object": "list", "data": [{"id": "gpt-b", "object": "model"}, {"id": "gpt-a"}]})
        if self.path == "/or/models":
            return self._json({"data": [{"id": "x/y", "name": "Y", "context_length": 8192,
                                         "pricing": {"prompt": "1", "completion": "2"}}]})
        self._json({"error": "no route"}, 404)

    def do_POST(self):
        body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
        SEEN.append((self.path, dict(self.headers), body))
        prompt = body.get("input") or (body.get("messages") or [{}])[0].get("content") or \
            body["contents"][0]["parts"][0]["text"]
        if "fail" in prompt:
            return self._json({"error": "boom"}, 500)
        words = ["echo:", " ", prompt]
        if self.path.startswith("/oa/responses"):
            if body.get("stream"):
                return self._sse([": keep-alive", "event: response.created", "data: {not json"] +
                                 [f"data: {json.dumps({'type': 'response.output_text.delta', 'delta': w})}"
                                  for w in words] + ["data: {\"type\": \"response.completed\"}", "data: [DONE]",
                                                     "data: " + json.dumps({"type": "response.output_text.delta",
                                                                            "delta": "AFTER-DONE"})])
            return self._json({"id": "r1", "output": [
                {"type": "reasoning"},
                {"type": "message", "content": [{"type": "output_text", "text": "".join(words)},
                                                {"type": "refusal", "text": "x"}]}]})
        if self.path.startswith("/an/messages"):
            if body.get("stream"):
                return self._sse(["event: message_start", "data: {\"type\": \"message_start\"}"] +
                                 [f"data: {json.dumps({'type': 'content_block_delta', 'delta': {'type': 'text_delta', 'text': w}})}"
                                  for w in words] +
                                 ["data: {\"type\": \"content_block_delta\", \"delta\": {\"type\": \"input_json_delta\"}}",
                                  "data: {\"type\": \"message_stop\"}"])
            return self._json({"content": [{"type": "text", "text": "".join(words)}]})
        if self.path.startswith("/go/models/"):
            if "streamGenerateContent" in self.path:
                return self._sse([f"data: {json.dumps({'candidates': [{'content': {'parts': [{'text': w}]}}]})}"
                                  for w in words] + ["data: {\"candidates\": []}"])
            return self._json({"candidates": [{"content": {"parts": [{"text": "".join(words)}]}}]})
        self._json({"error": "no route"}, 404)


@pytest.fixture(scope="module")
def server():
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _H)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    base = f"http://127.0.0.1:{srv.server_address[1]}"
    yield base
    srv.shutdown()


def _providers(base):
    return [OpenAIProvider("gpt-5.2-2025-12-11", "k-oa", base + "/oa"),
            AnthropicProvider("claude-sonnet-4-5", "k-an", base + "/an"),
            GoogleProvider("gemini-3-pro-preview", "k-go", base + "/go")]


def test_stream_and_query_all_three(server):
    for p in _providers(server):
        chunks = []
        r = p.query_stream(Context.background(), Request(p.model, "hi there"), chunks.append)
        assert r.content == "echo: hi there" and "".join(chunks) == r.content, (p.provider_name, r.content)
        assert r.provider == p.provider_name and r.model == p.model and r.latency_ns > 0
        q = p.query(Context.background(), Request(p.model, "hi"))
        assert q.content == "echo: hi"


def test_wire_format(server):
    SEEN.clear()
    oa, an, go = _providers(server)
    oa.query_stream(Context.background(), Request(oa.model, "p"), None)
    an.query_stream(Context.background(), Request(an.model, "p"), None)
    go.query_stream(Context.background(), Request(go.model, "p"), None)
    (p1, h1, b1), (p2, h2, b2), (p3, h3, b3) = SEEN
    assert p1 == "/oa/responses" and h1["Authorization"] == "Bearer k-oa"
    assert b1 == {"model": "gpt-5.2-2025-12-11", "input": "p", "stream": True}
    assert p2 == "/an/messages" and h2["x-api-key"] == "k-an" and h2["anthropic-version"] == "2023-06-01"
    assert b2 == {"model": "claude-sonnet-4-5", "max_tokens": 4096, "messages": [{"role": "user", "content": "p"}],
                  "stream": True}
    assert p3 == "/go/models/gemini-3-pro-preview:streamGenerateContent?key=k-go&alt=sse"
    assert b3 == {"contents": [{"parts": [{"text": "p"}]}]}


def test_errors(server, monkeypatch):
    oa = _providers(server)[0]
    with pytest.raises(RemoteError, match=r"API error \(status 500\): .*boom"):
        oa.query_stream(Context.background(), Request(oa.model, "please fail"), None)
    monkeypatch.delenv("OPENAI_API_KEY", raising=False)
    with pytest.raises(RemoteError, match="OPENAI_API_KEY environment variable required"):
        create("gpt-5.2-2025-12-11", "openai")


def test_cli_with_hosted_models(server, tmp_path):
    env = dict(os.environ, OPENAI_API_KEY="a", ANTHROPIC_API_KEY="b", GOOGLE_API_KEY="c",
               OPENAI_BASE_URL=server + "/oa", ANTHROPIC_BASE_URL=server + "/an", GOOGLE_BASE_URL=server + "/go")
    r = subprocess.run([sys.executable, "-m", "llm_consensus_amd", "--models",
                        "gpt-5.2-2025-12-11,claude-opus-4-5,gemini-3-pro-preview", "--judge", "stub-j", "--json",
                        "compare"], cwd=ROOT, env=env, capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    d = json.loads(r.stdout)
    got = {x["model"]: (x["provider"], x["content"]) for x in d["responses"]}
    assert got == {"gpt-5.2-2025-12-11": ("openai", "echo: compare"), "claude-opus-4-5": ("anthropic", "echo: compare"),
                   "gemini-3-pro-preview": ("google", "echo: compare")}
    # missing key -> initialization error naming the model (main.go:409)
    env.pop("GOOGLE_API_KEY")
    r = subprocess.run([sys.executable, "-m", "llm_consensus_amd", "--models", "gemini-3-pro-preview", "--judge", "stub-j",
                        "x"], cwd=ROOT, env=env, capture_output=True, timeout=120)
    assert r.returncode == 1
    assert b"error: initializing provider for gemini-3-pro-preview: GOOGLE_API_KEY environment variable required" in r.stderr


def test_registry_sync_remote_sources(server, tmp_path):
    env = dict(os.environ, OPENAI_API_KEY="k", OPENAI_BASE_URL=server + "/oa", OPENROUTER_BASE_URL=server + "/or")
    r = subprocess.run([sys.executable, "-m", "llm_consensus_amd.registry_sync", "-local=false", "-hf-cache=false"],
                       cwd=ROOT, env=env, capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    recs = json.loads(r.stdout)
    assert recs == [{"source": "openai", "id": "gpt-a"}, {"source": "openai", "id": "gpt-b"},
                    {"source": "openrouter", "id": "x/y", "name": "Y", "context_length": 8192,
                     "pricing": {"prompt": "1", "completion": "2", "request": "", "image": ""}}]
    env.pop("OPENAI_API_KEY")
    r = subprocess.run([sys.executable, "-m", "llm_consensus_amd.registry_sync", "-local=false", "-hf-cache=false"],
                       cwd=ROOT, env=env, capture_output=True, timeout=120)
    assert r.returncode == 0 and b"openai: OPENAI_API_KEY not set" in r.stderr
