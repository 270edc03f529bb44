"""Local MI355X provider: the replacement for the remote OpenAI/Anthropic/Google adapters
(reference ``internal/provider/{openai,anthropic,google}.go``).

``LocalBackend`` places every local model of the run on the node's GPUs (``parallel/placement``),
spawns one worker process per used GPU (``runtime/worker``), and multiplexes their token streams.
``LocalProvider.query_stream`` keeps the reference contract: incremental text chunks go to the
callback, the returned ``content`` is their concatenation, ``latency`` spans request → end of
stream. The "transport" is a pipe to the worker instead of HTTPS+SSE; cancellation/deadline
are checked between token batches and propagate to the worker (the engine stops within one
decode graph replay, a few ms).

Judge sessions: the judge prompt is rendered as header + per-response blocks in
completion order + trailer, so the judge engine prefills the header at run start and each block
as its response completes (``open_session`` / ``extend_session``); at synthesis time only the
last block's remainder and the trailer are prefilled before decoding.
"""

from __future__ import annotations

import itertools
import os
import queue
import socket
import threading
import time
import zlib
from typing import Dict, List, Optional

from ..catalog import PROVIDER_LOCAL, ModelSpec
from ..context import Context, ContextError
from ..parallel.placement import (HBM_BYTES, USABLE_FRACTION, ModelDemand, alone_plan, default_gpus, describe,
                                  fused_ar_plan, solve)
from ..utils import trace as tracing
from ..utils.tokenizer import tokenizer_for
from .base import Request, Response, StreamCallback

DEFAULT_MAX_TOKENS = 4096
RESPONDER_CONTEXT = 16384
JUDGE_CONTEXT = 131072
KV_BLOCK = 64  # tokens per paged-KV block (EngineConfig.block_size)


def kv_pool_blocks(placement, specs, ctx: Dict[str, int], seqs: Dict[str, int],
                   hbm_bytes: int = HBM_BYTES) -> Dict[str, int]:
    """Paged-KV pool per engine, in blocks. An engine asks for ``seqs[m]`` full contexts (every live
    sequence at max_context); when the engines of a GPU ask for more than its HBM left after their
    weights, each gets a share proportional to its ask but never less than one full context (what
    placement reserved). Sequences take blocks as they grow, so a pool smaller than the ask only
    limits how many LONG sequences can be live at once (a request that cannot reserve its blocks
    fails with an engine error) — e.g. 16 judge sessions at a 131k context would ask for 290 GB."""
    free = {}
    for m, gs in placement.gpus.items():
        for g in gs:
            free.setdefault(g, hbm_bytes * USABLE_FRACTION)
            free[g] -= specs[m].config.weight_bytes() / len(gs)
    per_tok = {m: specs[m].config.kv_bytes_per_token() / len(gs) for m, gs in placement.gpus.items()}
    out = {}
    for m, gs in placement.gpus.items():
        ask = seqs[m] * ctx[m] * per_tok[m]
        floor = ctx[m] * per_tok[m]
        scale = 1.0
        for g in gs:
            asks = sum(seqs[o] * ctx[o] * per_tok[o] for o, og in placement.gpus.items() if g in og)
            scale = min(scale, max(0.0, free[g]) / asks if asks > 0 else 1.0)
        tokens = max(floor, ask * min(1.0, scale)) / per_tok[m] if per_tok[m] else ctx[m] * seqs[m]
        out[m] = int(tokens) // KV_BLOCK + 2 * seqs[m] + 2
    return out


class LocalError(Exception):
    pass


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Worker:
    def __init__(self, backend: "LocalBackend", gpu: int, conn, proc):
        self.backend = backend
        self.gpu = gpu
        self.conn = conn
        self.proc = proc
        self.send_lock = threading.Lock()
        self.ready = threading.Event()
        self.fatal: Optional[str] = None
        self.info = None
        self.t = threading.Thread(target=self._recv_loop, daemon=True, name=f"worker-rx:{gpu}")
        self.t.start()

    def send(self, msg) -> None:
        with self.send_lock:
            self.conn.send(msg)

    def _recv_loop(self) -> None:
        while True:
            try:
                msg = self.conn.recv()
            except (EOFError, OSError):
                self.fatal = self.fatal or f"worker gpu{self.gpu} exited"
                self.ready.set()
                self.backend._worker_died(self)
                return
            kind = msg[0]
            if kind == "ready":
                self.info = msg[1]
                self.ready.set()
            elif kind == "fatal":
                self.fatal = msg[1]
                self.ready.set()
            elif kind == "trace":
                tracing.add_events(msg[1])
            else:
                self.backend._deliver(msg)


# = ops.GEMV_MAX_M / ops.MOE_GEMVM_MAX_TOKENS (not imported: the driver process stays torch-free;
# tests/test_placement.py checks they agree)
DECODE_ROWS_MAX, MOE_DECODE_ROWS_MAX = 32, 16


def max_decode_rows(cfg) -> int:
    """Decode rows one engine batches per step: the MFMA weight-streaming form takes 32 token rows
    (two 16-token column groups); batched MoE decode groups (row, expert) pairs of <= 16 tokens."""
    return MOE_DECODE_ROWS_MAX if cfg.is_moe else DECODE_ROWS_MAX


class LocalBackend:
    """Owns the worker processes of one run and routes requests to them."""

    def __init__(self, specs: List[ModelSpec], judge: Optional[str] = None, gpus: Optional[List[int]] = None,
                 trace: bool = False, counts: Optional[Dict[str, int]] = None,
                 max_context: Optional[Dict[str, int]] = None, start_timeout: float = 1800.0,
                 pins: Optional[Dict[str, List[int]]] = None, judge_tp: int = 0, concurrency: int = 1):
        """``concurrency``: consensus requests served at once (the server): each engine gets decode
        rows for that many requests (replica batching, up to 4 rows) and KV for their sequences
        plus one judge session per request."""
        import multiprocessing as mp

        self.specs = {s.name: s for s in specs}
        self.judge = judge
        force_cpu = os.environ.get("LLMC_DEVICE", "") == "cpu"
        # CPU workers (tests): LLMC_CPU_WORKERS=k spreads the models over k worker processes
        n_cpu = max(1, int(os.environ.get("LLMC_CPU_WORKERS", "1")))
        gpu_ids = [-(i + 1) for i in range(n_cpu)] if force_cpu else default_gpus(gpus)
        if not gpu_ids:
            raise LocalError("no ROCm GPU visible (set LLMC_DEVICE=cpu to run local models on the CPU)")
        self._queues: Dict[int, "queue.Queue"] = {}
        self._rid_model: Dict[int, str] = {}
        self._qlock = threading.Lock()
        self._bcast_lock = threading.Lock()
        self._ids = itertools.count(1)
        self.closed = False

        if judge_tp > 1 and judge in self.specs and not (pins and judge in pins):
            # the judge phase follows the fan-out, when the responders' GPUs are idle: shard the
            # judge over the first judge_tp of them (co-located on its own streams)
            if judge_tp > len(gpu_ids):
                raise LocalError(f"--judge-tp {judge_tp} needs {judge_tp} GPUs, {len(gpu_ids)} available")
            pins = dict(pins or {})
            pins[judge] = list(gpu_ids[:judge_tp])
        demands = []
        self._ctx = {}
        for s in specs:
            c = s.config
            ctx_len = (max_context or {}).get(s.name) or min(c.max_position,
                                                             JUDGE_CONTEXT if s.name == judge else RESPONDER_CONTEXT)
            self._ctx[s.name] = ctx_len
            if pins and s.name in pins:
                tp = len(pins[s.name])
            else:
                tp = 1 if force_cpu else min(c.default_tp, len(gpu_ids))
            demands.append(ModelDemand(s.name, c.weight_bytes(), c.kv_bytes_per_token() * ctx_len, tp, s.name == judge))
        if force_cpu and not pins:
            from ..parallel.placement import Placement

            # CPU workers: round-robin (tests); with --placement pins, the solver as on GPUs (CPU TP
            # groups run over gloo, so config-4/5 style TP judges are testable without GPUs)
            self.placement = Placement({s.name: [gpu_ids[i % len(gpu_ids)]] for i, s in enumerate(specs)})
        else:
            self.placement = solve(demands, gpu_ids, pins=pins)
        trace_on = trace
        used = self.placement.used_gpus()
        groups = [(m, sorted(g)) for m, g in self.placement.gpus.items() if len(g) > 1]
        dist_info = None
        rank_of = {g: i for i, g in enumerate(used)}
        port = _free_port() if groups else 0
        ctxm = mp.get_context("spawn")
        self.workers: Dict[int, _Worker] = {}
        from ..runtime.worker import worker_main

        conc = max(1, concurrency)
        seqs = {}
        for m in self.placement.gpus:
            # responder rows: one per --models entry per request in flight; a judge-only engine
            # needs a session per request (and a row for plain queries)
            n = (counts or {}).get(m, 0 if m == judge else 1) * conc
            sess = conc if m == judge else 0
            seqs[m] = (n, sess)
        kv_blocks = kv_pool_blocks(self.placement, self.specs, self._ctx,
                                   {m: max(1, n) + sess for m, (n, sess) in seqs.items()})
        # the engines that decode during the fan-out (a judge named in --models is one of them)
        responders = [m for m, (n, _) in seqs.items() if n > 0]
        fused = fused_ar_plan(self.placement.gpus, judge, conc, responders)
        alone = alone_plan(self.placement.gpus, judge, conc, responders)
        for g in used:
            models = []
            for m, gs in self.placement.gpus.items():
                if g in gs:
                    s = self.specs[m]
                    n, sess = seqs[m]
                    models.append({"name": m, "family": s.family, "seed": s.seed, "max_context": self._ctx[m],
                                   "checkpoint": s.config.checkpoint, "kv_blocks": kv_blocks[m],
                                   # decode rows per step: up to 32 on the weight-streaming
                                   # GEMV / MFMA form (MoE: 16, pairs grouped by expert)
                                   "max_batch": max(1, min(max_decode_rows(s.config), max(n, sess))),
                                   "max_seqs": max(1, n) + sess,
                                   # TP: the all-reduce in the row-parallel GEMVs' epilogue unless
                                   # an engine decoding at the same time shares its GPUs
                                   "fused_ar": fused[m],
                                   # no other engine decodes on its GPUs meanwhile: the lone-engine
                                   # launch forms (ops.attn_oproj_min_chunk)
                                   "alone": alone[m]})
            if groups:
                dist_info = {"port": port, "rank": rank_of[g], "world": len(used),
                             "groups": [(m, [rank_of[x] for x in gs]) for m, gs in groups]}
            a, b = ctxm.Pipe(duplex=True)
            p = ctxm.Process(target=worker_main, args=(g, b, models, dist_info, trace_on), daemon=True,
                             name=f"llmc-worker-gpu{g}")
            p.start()
            b.close()
            self.workers[g] = _Worker(self, g, a, p)
        tracing.instant("workers_spawned", cat="startup", n=len(self.workers))
        deadline = time.monotonic() + start_timeout
        for w in self.workers.values():
            if not w.ready.wait(max(0.0, deadline - time.monotonic())):
                self.close()
                raise LocalError(f"worker gpu{w.gpu} did not start in {start_timeout:.0f}s")
            if w.fatal:
                msg = w.fatal
                self.close()
                raise LocalError(msg.splitlines()[0])
        tracing.instant("placement", plan=describe(self.placement))

    # -- routing ----------------------------------------------------------------------------------
    def _workers_for(self, model: str) -> List[_Worker]:
        return [self.workers[g] for g in self.placement.gpus[model]]

    def _new_request(self, model: str = "") -> (int, "queue.Queue"):
        rid = next(self._ids)
        q: "queue.Queue" = queue.Queue()
        with self._qlock:
            self._queues[rid] = q
            self._rid_model[rid] = model
        return rid, q

    def _end_request(self, rid: int) -> None:
        with self._qlock:
            self._queues.pop(rid, None)
            self._rid_model.pop(rid, None)

    def _deliver(self, msg) -> None:
        with self._qlock:
            q = self._queues.get(msg[1])
        if q is not None:
            q.put(msg)

    def _worker_died(self, w: _Worker) -> None:
        """Liveness: a dead worker fails the requests of the models it hosts
        (every rank of a TP group counts); models on other workers keep running."""
        hosted = {m for m, gs in self.placement.gpus.items() if w.gpu in gs} if self.placement else None
        with self._qlock:
            qs = [(rid, q) for rid, q in self._queues.items()
                  if hosted is None or not self._rid_model.get(rid) or self._rid_model[rid] in hosted]
        for rid, q in qs:
            q.put(("error", rid, w.fatal or "worker died"))

    def broadcast(self, model: str, msg) -> None:
        """Send ``msg`` to every worker hosting ``model``. Atomic across workers: concurrent
        callers (the runner's per-model threads, the judge session) must reach every rank of a TP
        group in ONE order, or the ranks would batch / prefill different requests."""
        with self._bcast_lock:
            for w in self._workers_for(model):
                if w.fatal:
                    raise LocalError(w.fatal.splitlines()[0])
                w.send(msg)

    def provider(self, name: str) -> "LocalProvider":
        return LocalProvider(self, name)

    def collect_traces(self) -> None:
        for w in self.workers.values():
            try:
                w.send(("trace",))
            except Exception:  # noqa: BLE001
                pass
        time.sleep(0.2)

    def close(self) -> None:
        if self.closed:
            return
        self.closed = True
        for w in self.workers.values():
            try:
                w.send(("shutdown",))
            except Exception:  # noqa: BLE001
                pass
        for w in self.workers.values():
            w.proc.join(timeout=60)
            if w.proc.is_alive():
                w.proc.terminate()
                w.proc.join(timeout=10)


class LocalProvider:
    """Provider facade for one local model (``query_stream`` contract of provider.go:13-21)."""

    provider_name = PROVIDER_LOCAL

    def __init__(self, backend: LocalBackend, model: str):
        self.backend = backend
        self.model = model
        self.spec = backend.specs[model]
        self.tok = tokenizer_for(self.spec.config)
        self._sess_lock = threading.Lock()
        self._session: Optional["JudgeSession"] = None

    # -- helpers ------------------------------------------------------------------------------------
    def _params(self, req: Request, prompt_len: int) -> dict:
        ctx_cap = self.backend._ctx[self.model] - prompt_len - 16
        if ctx_cap < 1:
            raise LocalError(f"prompt of {prompt_len} tokens exceeds {self.model} context {self.backend._ctx[self.model]}")
        mt = min(req.max_tokens or DEFAULT_MAX_TOKENS, ctx_cap)
        seed = req.seed if req.seed is not None else (zlib.crc32(self.model.encode()) & 0x7FFFFFFF)
        return {"max_tokens": int(mt), "temperature": 1.0 if req.temperature is None else float(req.temperature),
                "top_p": 1.0 if req.top_p is None else float(req.top_p), "top_k": int(req.top_k or 0),
                "seed": int(seed), "stop_on_eos": True if req.stop_on_eos is None else bool(req.stop_on_eos)}

    def _stream(self, ctx: Context, rid: int, q: "queue.Queue", callback: Optional[StreamCallback], t0: int,
                prompt_tokens: int) -> Response:
        dec = self.tok.stream_decoder()
        parts: List[str] = []
        ntok = 0
        ttft = 0
        try:
            while True:
                try:
                    msg = q.get(timeout=0.05)
                except queue.Empty:
                    if ctx.done():
                        self.backend.broadcast(self.model, ("cancel", rid))
                        raise ContextError(ctx.err())
                    continue
                kind = msg[0]
                if kind == "tokens":
                    if not ttft:
                        ttft = time.monotonic_ns() - t0
                    ntok += len(msg[2])
                    hook = getattr(callback, "tokens_hook", None)
                    if hook is not None:
                        hook(len(msg[2]))
                    chunk = dec.push(msg[2])
                    if chunk:
                        parts.append(chunk)
                        if callback is not None:
                            callback(chunk)
                elif kind == "done":
                    break
                elif kind == "error":
                    raise LocalError(msg[2])
            tail = dec.flush()
            if tail:
                parts.append(tail)
                if callback is not None:
                    callback(tail)
        finally:
            self.backend._end_request(rid)
        return Response(model=self.model, content="".join(parts), provider=self.provider_name,
                        latency_ns=time.monotonic_ns() - t0, prompt_tokens=prompt_tokens, output_tokens=ntok,
                        ttft_ns=ttft)

    # -- Provider API -------------------------------------------------------------------------------
    def query(self, ctx: Context, req: Request) -> Response:
        return self.query_stream(ctx, req, None)

    def query_stream(self, ctx: Context, req: Request, callback: Optional[StreamCallback]) -> Response:
        t0 = time.monotonic_ns()
        ids = self.tok.encode_prompt(req.prompt)
        params = self._params(req, len(ids))
        rid, q = self.backend._new_request(self.model)
        with tracing.span("query", cat="driver", model=self.model, prompt_tokens=len(ids)):
            self.backend.broadcast(self.model, ("generate", rid, self.model, ids, params))
            return self._stream(ctx, rid, q, callback, t0, len(ids))

    # -- judge sessions (incremental prefill) ---------------------------------------------------------
    def new_session(self, header: str) -> "JudgeSession":
        """A judge KV session of its own (the server runs one per concurrent request)."""
        return JudgeSession(self, header)

    def open_session(self, header: str) -> None:
        """The provider's default session (one consensus run at a time: the CLI)."""
        with self._sess_lock:
            self.close_session()
            self._session = JudgeSession(self, header)

    def extend_session(self, text: str) -> None:
        s = self._session
        if s is not None:
            s.extend(text)

    def close_session(self) -> None:
        s = self._session
        self._session = None
        if s is not None:
            s.close()

    def query_stream_session(self, ctx: Context, req: Request, callback: Optional[StreamCallback]) -> Response:
        with self._sess_lock:
            s = self._session
            self._session = None
        if s is None:
            return self.query_stream(ctx, req, callback)
        return s.finish(ctx, req, callback)

    def close(self) -> None:
        self.close_session()
        self.backend.close()


class JudgeSession:
    """A judge prompt being prefilled incrementally on the judge engine: the
    header at open, each response block as it completes (``extend``), then ``finish`` prefills
    what is left and decodes. Sessions are independent (own engine sequence), so concurrent
    consensus requests each keep their own."""

    def __init__(self, provider: LocalProvider, header: str):
        self.provider = provider
        self._lock = threading.Lock()
        self.sid = next(provider.backend._ids)
        ids = provider.tok.prompt_prefix_ids(header)
        self.text = header
        self.ids = list(ids)
        self.open = True
        provider.backend.broadcast(provider.model, ("sess_open", self.sid, provider.model, ids))

    def extend(self, text: str) -> None:
        with self._lock:
            if not self.open:
                return
            ids = self.provider.tok.encode(text)
            self.text += text
            self.ids.extend(ids)
            self.provider.backend.broadcast(self.provider.model, ("sess_extend", self.sid, ids))

    def close(self) -> None:
        with self._lock:
            if not self.open:
                return
            self.open = False
        try:
            self.provider.backend.broadcast(self.provider.model, ("sess_close", self.sid))
        except Exception:  # noqa: BLE001
            pass

    def finish(self, ctx: Context, req: Request, callback: Optional[StreamCallback]) -> Response:
        """Decode the judge answer for ``req.prompt``, whose prefix this session holds.

        The prompt is tokenized whole (exactly as ``query_stream`` would) and matched against the
        ids already prefilled: only the unmatched tail is prefilled, after truncating the session
        to the common prefix (tokenizers that are not segment-stable, chat templates)."""
        p = self.provider
        with self._lock:
            live = self.open
            self.open = False
        if not live or not req.prompt.startswith(self.text):
            if live:
                p.backend.broadcast(p.model, ("sess_close", self.sid))
            return p.query_stream(ctx, req, callback)
        t0 = time.monotonic_ns()
        full = p.tok.encode_prompt(req.prompt)
        done = self.ids
        cp = 0
        n = min(len(done), len(full))
        while cp < n and done[cp] == full[cp]:
            cp += 1
        if cp == len(full):  # keep at least one token to prefill (its logits start the decode)
            cp -= 1
        rest = full[cp:]
        params = p._params(req, len(full))
        rid, q = p.backend._new_request(p.model)
        with tracing.span("judge_session_finish", cat="driver", model=p.model, rest_tokens=len(rest),
                          reused_tokens=cp):
            p.backend.broadcast(p.model, ("sess_generate", self.sid, rid, rest, params, cp))
            return p._stream(ctx, rid, q, callback, t0, len(full))
