"""Consensus serving daemon: warm engines, concurrent requests, HTTP + SSE.

The reference is a one-shot CLI (``cmd/llm-consensus/main.go``): every run pays process start,
and with local engines that means weight load/init and HIP-graph capture (≈18 s of the 47.7 s CLI
wall time in BASELINE.md §2.1). The server keeps the node's engines resident and answers
consensus requests with the reference's exact semantics — best-effort fan-out in completion
order (``internal/runner``), single-response passthrough and judge template
(``internal/consensus``), the ``result.json`` schema (``internal/output``) — over HTTP:

  GET  /healthz            {"status": "ok", "models": [...], "judge": "..."}
  GET  /v1/models          served models and their providers
  POST /v1/consensus       {"prompt": "...", "models": [...], "judge": "...", "max_tokens": N,
                            "temperature": T, "top_p": P, "top_k": K, "seed": S, "timeout": SEC,
                            "stream": false}
       stream=false: 200 + the Go-compatible result JSON (byte-identical to result.json)
       stream=true:  200 text/event-stream: model_start / chunk / tokens / model_done /
                     model_error / judge_start / judge_chunk / result (the result JSON) / error

Concurrent requests share the engines: requests for the same engine are batched into one decode
(replica batching: up to 4 rows read each weight once, runtime/worker.py), each request keeps its
own incrementally prefilled judge session (provider/local.JudgeSession), and judge sessions that
finish together decode as one batch. ``--concurrency`` sizes the engines' decode rows and KV for
that many requests in flight; more requests wait for a slot.

  python -m llm_consensus_amd.server --models llama-3-8b@0,llama-3-8b@1 --judge llama-3-8b@judge \\
      --port 8080 --concurrency 4
  llm-consensus --server http://127.0.0.1:8080 --models llama-3-8b@0,llama-3-8b@1 "prompt"
"""

from __future__ import annotations

import argparse
import json
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, List, Optional

from .consensus import Judge, prompt_header, response_block
from .context import Context
from .output import Result, encode_result
from .provider.base import Request, Response
from .runner import Callbacks, Runner

EventFn = Callable[[str, dict], None]


class BadRequest(Exception):
    pass


class ServiceError(Exception):
    pass


class _SessionJudge:
    """Provider facade binding one request's judge session (``consensus.Judge`` looks for
    ``close_session`` / ``query_stream_session`` on its provider); keeps the judge's Response
    (token counts, latency) for the caller."""

    def __init__(self, provider, session):
        self.provider = provider
        self.session = session
        self.response: Optional[Response] = None

    def close_session(self) -> None:
        if self.session is not None:
            self.session.close()

    def query_stream_session(self, ctx, req, callback):
        if self.session is None:
            return self.query_stream(ctx, req, callback)
        self.response = self.session.finish(ctx, req, callback)
        return self.response

    def query_stream(self, ctx, req, callback):
        self.response = self.provider.query_stream(ctx, req, callback)
        return self.response


class ConsensusService:
    """Engines for ``models`` + ``judge`` placed once; ``run`` serves one consensus request and
    is safe to call from many threads at once."""

    def __init__(self, models: List[str], judge: str, gpus: str = "", placement: str = "", judge_tp: int = 0,
                 concurrency: int = 4, timeout: float = 120.0, max_tokens: int = 0, temperature: float = 1.0,
                 top_p: float = 1.0, top_k: int = 0, seed: int = 0):
        from .cli import Config, init_registry

        self.responders = list(dict.fromkeys(models))
        self.judge = judge
        self.timeout = timeout
        self.concurrency = max(1, concurrency)
        self.defaults = dict(max_tokens=max_tokens, temperature=temperature, top_p=top_p, top_k=top_k, seed=seed)
        cfg = Config(models=self.responders, judge=judge, file="", output="", data_dir="", timeout=timeout,
                     prompt="", quiet=True, json=True, no_save=True, max_tokens=max_tokens,
                     temperature=temperature, top_p=top_p, top_k=top_k, seed=seed, gpus=gpus, trace=False,
                     placement=placement, judge_tp=judge_tp)
        self.registry = init_registry(cfg, concurrency=self.concurrency)
        self.served = self.registry.models()
        self._slots = threading.BoundedSemaphore(self.concurrency)
        self.stats = {"requests": 0, "failed": 0, "in_flight": 0}
        self._stats_lock = threading.Lock()

    def close(self) -> None:
        self.registry.close()

    def _param(self, body: dict, key: str, typ, default):
        v = body.get(key, None)
        if v is None:
            return default
        try:
            if typ is int and (isinstance(v, bool) or (isinstance(v, float) and not v.is_integer())):
                raise ValueError
            return typ(v)
        except (TypeError, ValueError):
            raise BadRequest(f"{key}: expected {typ.__name__}, got {v!r}") from None

    def parse(self, body: dict) -> dict:
        """Validate a request body (the reference's bootstrap checks, main.go:332-339, 395-426)."""
        if not isinstance(body, dict):
            raise BadRequest("request body must be a JSON object")
        prompt = body.get("prompt")
        if not isinstance(prompt, str) or prompt == "":
            raise BadRequest("no prompt provided: \"prompt\" must be a non-empty string")
        models = body.get("models", None)
        if models is None:
            models = list(self.responders)
        elif isinstance(models, str):
            models = [m.strip() for m in models.split(",")]
        if not isinstance(models, list) or not models or not all(isinstance(m, str) for m in models):
            raise BadRequest("models: expected a non-empty list of model names")
        judge = body.get("judge") or self.judge
        for m in models + [judge]:
            if m not in self.served:
                raise BadRequest(f"initializing provider for {m}: unknown model {json.dumps(m)}; "
                                 f"available models: [{' '.join(self.served)}]")
        d = self.defaults
        return {
            "prompt": prompt, "models": models, "judge": judge,
            "timeout": self._param(body, "timeout", float, self.timeout),
            "max_tokens": self._param(body, "max_tokens", int, d["max_tokens"]),
            "temperature": self._param(body, "temperature", float, d["temperature"]),
            "top_p": self._param(body, "top_p", float, d["top_p"]),
            "top_k": self._param(body, "top_k", int, d["top_k"]),
            "seed": self._param(body, "seed", int, d["seed"]),
            "stream": bool(body.get("stream", False)),
        }

    def run(self, ctx: Context, req: dict, emit: Optional[EventFn] = None) -> Result:
        """One consensus round (cli._run_with_registry without the UI/persistence)."""
        def ev(name: str, data: dict) -> None:
            if emit is not None:
                emit(name, data)

        with self._slots:
            with self._stats_lock:
                self.stats["requests"] += 1
                self.stats["in_flight"] += 1
            try:
                return self._run(ctx, req, ev)
            except Exception:
                with self._stats_lock:
                    self.stats["failed"] += 1
                raise
            finally:
                with self._stats_lock:
                    self.stats["in_flight"] -= 1

    def _run(self, ctx: Context, req: dict, ev: EventFn) -> Result:
        prompt, models, judge_name = req["prompt"], req["models"], req["judge"]
        tmpl = Request(model="", prompt="", max_tokens=req["max_tokens"] or None, temperature=req["temperature"],
                       top_p=req["top_p"], top_k=req["top_k"] or None, seed=req["seed"] or None,
                       stop_on_eos=req.get("stop_on_eos"))
        jp = self.registry.get(judge_name)
        session = None
        if hasattr(jp, "new_session") and len(models) > 1 and judge_name == self.judge:
            session = jp.new_session(prompt_header(prompt))

        def on_response(r: Response) -> None:
            if session is not None:
                session.extend(response_block(r))
            ev("model_done", {"model": r.model, "provider": r.provider, "latency_ms": r.latency_ms,
                              "output_tokens": r.output_tokens})

        runner = Runner(self.registry, req["timeout"], tmpl).with_callbacks(Callbacks(
            on_model_start=lambda m: ev("model_start", {"model": m}),
            on_model_stream=lambda m, c: ev("chunk", {"model": m, "text": c}),
            on_model_tokens=lambda m, n: ev("tokens", {"model": m, "n": n}),
            on_model_error=lambda m, e: ev("model_error", {"model": m, "error": str(e)}),
            on_model_response=on_response,
        ))
        try:
            result = runner.run(ctx, models, prompt)
        except Exception as e:  # noqa: BLE001
            if session is not None:
                session.close()
            raise ServiceError(f"running queries: {e}") from None
        ev("judge_start", {"judge": judge_name, "responses": len(result.responses)})
        jw = _SessionJudge(jp, session) if session is not None or hasattr(jp, "new_session") else None
        judge = Judge(jw if jw is not None else jp, judge_name, tmpl)
        try:
            consensus = judge.synthesize_stream(ctx.with_timeout(req["timeout"]), prompt, result.responses,
                                                lambda c: ev("judge_chunk", {"text": c}))
        except Exception as e:  # noqa: BLE001
            raise ServiceError(f"consensus synthesis: {e}") from None
        if jw is not None and jw.response is not None:
            ev("judge_done", {"output_tokens": jw.response.output_tokens, "prompt_tokens": jw.response.prompt_tokens,
                              "latency_ms": jw.response.latency_ms})
        return Result(prompt=prompt, responses=result.responses, consensus=consensus, judge=judge_name,
                      warnings=result.warnings, failed_models=result.failed_models)


def _sse(name: str, payload: str) -> bytes:
    lines = payload.split("\n")
    if lines and lines[-1] == "":
        lines.pop()
    return ("event: " + name + "\n" + "".join("data: " + ln + "\n" for ln in lines) + "\n").encode("utf-8",
                                                                                                   "surrogateescape")


def make_handler(service: ConsensusService):
    class Handler(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"
        server_version = "llm-consensus-amd"

        def log_message(self, fmt, *args):  # noqa: A003 - quiet by default (the CLI owns stdout)
            if getattr(self.server, "verbose", False):
                sys.stderr.write("%s - %s\n" % (self.address_string(), fmt % args))

        def _send(self, code: int, body: bytes, ctype: str = "application/json") -> None:
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def _json(self, code: int, obj) -> None:
            self._send(code, (json.dumps(obj) + "\n").encode())

        def do_GET(self):  # noqa: N802
            if self.path == "/healthz":
                with service._stats_lock:
                    st = dict(service.stats)
                self._json(200, {"status": "ok", "models": service.served, "judge": service.judge,
                                 "concurrency": service.concurrency, **st})
            elif self.path == "/v1/models":
                out = []
                for m in service.served:
                    p = service.registry.get(m)
                    out.append({"id": m, "provider": getattr(p, "provider_name", "") or type(p).__name__,
                                "role": "judge" if m == service.judge else "responder"})
                self._json(200, {"models": out})
            else:
                self._json(404, {"error": f"no route {self.path}"})

        def do_POST(self):  # noqa: N802
            if self.path != "/v1/consensus":
                self._json(404, {"error": f"no route {self.path}"})
                return
            try:
                n = int(self.headers.get("Content-Length") or 0)
                body = json.loads(self.rfile.read(n) or b"null")
                req = service.parse(body)
            except (ValueError, BadRequest) as e:
                self._json(400, {"error": str(e)})
                return
            ctx = Context.background()
            if not req["stream"]:
                try:
                    res = service.run(ctx, req)
                except ServiceError as e:
                    self._json(502, {"error": str(e)})
                    return
                self._send(200, encode_result(res).encode("utf-8", "surrogateescape"))
                return
            # streaming: events are written by the runner's threads as they happen
            self.send_response(200)
            self.send_header("Content-Type", "text/event-stream")
            self.send_header("Cache-Control", "no-cache")
            self.send_header("Connection", "close")
            self.end_headers()
            self.close_connection = True
            lock = threading.Lock()

            def emit(name: str, data) -> None:
                payload = data if isinstance(data, str) else json.dumps(data)
                with lock:
                    if ctx.done():
                        return
                    try:
                        self.wfile.write(_sse(name, payload))
                        self.wfile.flush()
                    except OSError:  # client went away: cancel the request's generations
                        ctx.cancel()

            try:
                res = service.run(ctx, req, emit)
                emit("result", encode_result(res))
            except ServiceError as e:
                emit("error", {"error": str(e)})

    return Handler


class ConsensusServer(ThreadingHTTPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, addr, service: ConsensusService, verbose: bool = False):
        super().__init__(addr, make_handler(service))
        self.service = service
        self.verbose = verbose


def serve(service: ConsensusService, host: str = "127.0.0.1", port: int = 8080, verbose: bool = False,
          ready: Optional[Callable[[int], None]] = None) -> None:
    srv = ConsensusServer((host, port), service, verbose)
    if ready is not None:
        ready(srv.server_address[1])
    try:
        srv.serve_forever(poll_interval=0.2)
    finally:
        srv.server_close()


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="llm-consensus-server", description=__doc__.split("\n\n")[0])
    ap.add_argument("--models", required=True, help="comma-separated responder models to serve")
    ap.add_argument("--judge", default="llama-3-8b@judge")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--concurrency", type=int, default=4, help="consensus requests in flight (batched decode)")
    ap.add_argument("--timeout", type=float, default=120.0, help="default per-model timeout (s)")
    ap.add_argument("--max-tokens", type=int, default=0)
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--top-p", type=float, default=1.0)
    ap.add_argument("--top-k", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--gpus", default="")
    ap.add_argument("--placement", default="")
    ap.add_argument("--judge-tp", type=int, default=0)
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)
    t0 = time.monotonic()
    svc = ConsensusService([m.strip() for m in a.models.split(",") if m.strip()], a.judge, gpus=a.gpus,
                           placement=a.placement, judge_tp=a.judge_tp, concurrency=a.concurrency,
                           timeout=a.timeout, max_tokens=a.max_tokens, temperature=a.temperature, top_p=a.top_p,
                           top_k=a.top_k, seed=a.seed)

    def ready(port: int) -> None:
        sys.stderr.write(f"llm-consensus server: {len(svc.served)} models ready in {time.monotonic() - t0:.1f}s, "
                         f"listening on http://{a.host}:{port}\n")
        sys.stderr.flush()

    try:
        serve(svc, a.host, a.port, a.verbose, ready)
    except KeyboardInterrupt:
        pass
    finally:
        svc.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())


__all__ = ["ConsensusService", "ConsensusServer", "serve", "main", "BadRequest", "ServiceError"]
