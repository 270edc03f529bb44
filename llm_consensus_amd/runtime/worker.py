"""GPU worker process: one per GPU, hosting every engine placed on that GPU (T3).

Control plane (C6): a duplex pipe to the driver carrying commands and token-id streams.
  driver -> worker  ("generate", rid, model, prompt_ids, params)
                    ("sess_open", sid, model, ids) / ("sess_extend", sid, ids)
                    ("sess_generate", sid, rid, ids, params, keep) / ("sess_close", sid)
                    ("cancel", rid) / ("shutdown",)
  worker -> driver  ("ready", info) / ("fatal", msg)
                    ("tokens", rid, ids) / ("done", rid, stats) / ("error", rid, msg)
Each engine has its own thread, hipStream and FIFO work queue, so engines co-located on a GPU
(responders + judge, config 3) run concurrently, and requests for the same engine are BATCHED
into one decode (replica batching: up to ``max_batch`` rows share every weight read).
TP engines: every rank of the group runs the same command sequence (the driver sends each
command to all ranks in the same order); only TP rank 0 streams tokens back.
"""

from __future__ import annotations

import datetime
import os
import queue
import threading
import time
import traceback
from typing import Dict, List, Optional


def parse_faults(spec: str) -> Dict[str, tuple]:
    """Fault-injection hook: ``LLMC_FAULT="<model>:<stage>[:<k>],..."`` makes that
    model's engine fail — stage ``init`` (every request errors), ``prefill`` (before prefill),
    ``decode`` (after k streamed tokens, default 1) or ``crash`` (the whole worker process dies
    abruptly on the first request: liveness path). Used by tests to exercise the best-effort
    failure path (runner.go:73-83) with real engines."""
    out: Dict[str, tuple] = {}
    for item in filter(None, (x.strip() for x in (spec or "").split(","))):
        parts = item.rsplit(":", 2) if item.count(":") >= 2 else item.rsplit(":", 1)
        if len(parts) == 3 and not parts[2].isdigit():
            parts = [parts[0] + ":" + parts[1], parts[2]]
        model, stage = parts[0], parts[1]
        k = int(parts[2]) if len(parts) == 3 else 1
        if stage not in ("init", "prefill", "decode", "crash"):
            raise ValueError(f"LLMC_FAULT: unknown stage {stage!r} in {item!r}")
        out[model] = (stage, k)
    return out


class InjectedFault(RuntimeError):
    pass


_EMPTY = object()
# a TP group's host control rounds (TPGroup._ctrl_exchange) never wait this long on a live peer: the
# ranks meet them in lockstep; a peer stalled past it fails the request and breaks the group
CTRL_TIMEOUT = datetime.timedelta(seconds=float(os.environ.get("LLMC_CTRL_TIMEOUT_S", "30")))
BATCH_WINDOW_S = float(os.environ.get("LLMC_BATCH_WINDOW_MS", "5")) / 1000.0


class _Req:
    __slots__ = ("rid", "ids", "params", "ctx")

    def __init__(self, rid, ids, params, ctx):
        self.rid, self.ids, self.params, self.ctx = rid, ids, params, ctx


class _EngineHost:
    def __init__(self, name: str, engine, send, leader: bool, fault: Optional[tuple] = None, on_finished=None):
        self.name = name
        self.on_finished = on_finished  # rid -> None: the worker drops the request's context
        self.fault = fault
        self.engine = engine
        self.send = send
        self.leader = leader
        self.q: "queue.Queue" = queue.Queue()
        self.sessions: Dict[int, object] = {}
        self._stash = _EMPTY  # an item taken off the queue while batching, processed next
        # continuous batching (rows join/leave between graph replays) for single-GPU engines sized
        # for several requests (the server, duplicate --models entries); LLMC_CONTINUOUS=0 = off
        cont = (engine.ecfg.max_batch > 1 and engine.tp.size == 1
                and os.environ.get("LLMC_CONTINUOUS", "1") != "0")
        self.t = threading.Thread(target=self._loop_continuous if cont else self._loop, daemon=True,
                                  name=f"engine:{name}")
        self.t.start()

    def _emit(self, *msg) -> None:
        if self.leader:
            self.send(msg)

    def _loop(self) -> None:
        from ..engine import SamplingParams

        while True:
            item, self._stash = (self._stash, _EMPTY) if self._stash is not _EMPTY else (self.q.get(), _EMPTY)
            if item is None:
                return
            kind = item[0]
            # the requests this item answers for: the first one until the batch is gathered, so a
            # failure while gathering still replies to it (and never to a previous batch)
            batch = [item[1]] if kind == "gen" else [item[2]] if kind == "sess_generate" else []
            try:
                if kind == "gen":
                    # replica batching: gather the generate requests for this engine that arrive
                    # within the batching window (concurrent requests are issued within ~1 ms)
                    batch = [r[1] for r in self._gather(item, "gen")]
                    self._generate(batch, SamplingParams)
                elif kind == "sess_open":
                    _, sid, ids = item
                    seq = self.engine.new_sequence()
                    self.sessions[sid] = seq
                    if ids:
                        self.engine.prefill([seq], [ids], want_logits=False)
                elif kind == "sess_extend":
                    _, sid, ids = item
                    seq = self.sessions.get(sid)
                    if seq is not None and ids:
                        self.engine.prefill([seq], [ids], want_logits=False)
                elif kind == "sess_generate":
                    # concurrent judge sessions (server) finishing together decode as one batch
                    items = self._gather(item, "sess_generate")
                    batch = [it[2] for it in items]
                    seqs = []
                    try:
                        for _, sid, req, keep in items:
                            seq = self.sessions.pop(sid, None)
                            if seq is None:
                                raise RuntimeError(f"unknown judge session {sid}")
                            seqs.append(seq)
                            if keep < seq.length:  # drop the prefilled tail the full tokenization differs on
                                self.engine.truncate(seq, keep)
                        self._run(seqs, batch, [r.ids for r in batch], SamplingParams)
                    finally:
                        for seq in seqs:
                            self.engine.free_sequence(seq)
                elif kind == "sess_close":
                    seq = self.sessions.pop(item[1], None)
                    if seq is not None:
                        self.engine.free_sequence(seq)
            except Exception as e:  # noqa: BLE001 - engine-level failure = that request's error
                rids = [r.rid for r in batch]
                msg = f"{type(e).__name__}: {e}"
                if os.environ.get("LLMC_DEBUG"):
                    msg += "\n" + traceback.format_exc()
                for rid in rids:
                    self._emit("error", rid, msg)
            finally:
                if self.on_finished is not None and kind in ("gen", "sess_generate"):
                    for r in batch:
                        self.on_finished(r.rid)

    def _gather(self, first, kind: str) -> list:
        """``first`` plus the queued items of the same kind, up to the engine's decode rows; waits
        up to the batching window (LLMC_BATCH_WINDOW_MS, default 5 ms, engines with > 1 row only)
        for items still arriving. A different kind ends the batch and is processed next.

        TP engines: the window is timing-dependent, so only the leader applies it; it broadcasts
        the batch size over the group's control channel and every follower takes exactly that
        many items (the driver sends every command to all ranks in one order, so they are the
        same requests) — identical batch compositions on every rank."""
        items = [first]
        cap = self.engine.ecfg.max_batch
        tp = self.engine.tp
        if tp.size > 1 and tp.ctrl is not None and not tp.is_leader:
            n = tp.leader_decides(0, "batch")
            while len(items) < n:
                items.append(self.q.get())
            return items
        if cap > 1:
            self._window(items, kind, cap)
        if tp.size > 1 and tp.ctrl is not None:
            tp.leader_decides(len(items), "batch")
        return items

    def _window(self, items: list, kind: str, cap: int) -> None:
        deadline = time.monotonic() + BATCH_WINDOW_S
        while len(items) < cap:
            try:
                nxt = self.q.get(timeout=max(0.0, deadline - time.monotonic()))
            except queue.Empty:
                break
            if nxt is None or nxt[0] != kind:
                self._stash = nxt  # next in line: keeps the queue's order
                break
            items.append(nxt)

    # -- continuous batching -------------------------------------------------------------------
    def _loop_continuous(self) -> None:
        """Commands are taken between replays: generate requests and judge-session finishes wait
        in ``waiting`` and are prefilled + admitted into free decode rows as rows retire; session
        open/extend/close prefill at once (they are short and order-sensitive)."""
        from collections import deque

        from ..engine import SamplingParams
        from ..engine.batcher import ContinuousBatcher

        stage, k = self.fault or ("", 0)
        sent: Dict[int, int] = {}

        def on_tokens(row, ids):
            req = row.tag[0]
            if not row.tag[2]:
                row.tag[2] = time.monotonic_ns() - row.tag[1]
            if stage == "decode" and sent.get(req.rid, 0) + len(ids) >= k:
                raise InjectedFault(f"injected fault: {self.name} decode after {k} tokens")
            sent[req.rid] = sent.get(req.rid, 0) + len(ids)
            self._emit("tokens", req.rid, ids)

        bat = ContinuousBatcher(self.engine, on_tokens)
        waiting: "deque" = deque()
        stop = False

        def fail(req, e) -> None:
            msg = f"{type(e).__name__}: {e}"
            if os.environ.get("LLMC_DEBUG"):
                msg += "\n" + traceback.format_exc()
            self._emit("error", req.rid, msg)
            if self.on_finished is not None:
                self.on_finished(req.rid)

        while not stop or bat.rows:
            # 1. commands: block only when there is nothing to decode
            items = []
            if not bat.rows and not waiting and not stop:
                if self._stash is not _EMPTY:
                    items.append(self._stash)
                    self._stash = _EMPTY
                else:
                    items.append(self.q.get())
                if items[0] is not None and items[0][0] in ("gen", "sess_generate") and self.engine.ecfg.max_batch > 1:
                    # a burst of concurrent requests: let the rest arrive before the first prefill
                    time.sleep(BATCH_WINDOW_S)
            while True:
                try:
                    items.append(self.q.get_nowait())
                except queue.Empty:
                    break
            for item in items:
                if item is None:
                    stop = True
                    continue
                kind = item[0]
                try:
                    if kind == "gen":
                        waiting.append(("gen", item[1], None, 0))
                    elif kind == "sess_generate":
                        _, sid, req, keep = item
                        seq = self.sessions.pop(sid, None)
                        if seq is None:
                            fail(req, RuntimeError(f"unknown judge session {sid}"))
                        else:
                            waiting.append(("sess", req, seq, keep))
                    elif kind == "sess_open":
                        _, sid, ids = item
                        seq = self.engine.new_sequence()
                        self.sessions[sid] = seq
                        if ids:
                            self.engine.prefill([seq], [ids], want_logits=False)
                    elif kind == "sess_extend":
                        _, sid, ids = item
                        seq = self.sessions.get(sid)
                        if seq is not None and ids:
                            self.engine.prefill([seq], [ids], want_logits=False)
                    elif kind == "sess_close":
                        seq = self.sessions.pop(item[1], None)
                        if seq is not None:
                            self.engine.free_sequence(seq)
                except Exception:  # noqa: BLE001 - a session command failed: drop the session, so its
                    if os.environ.get("LLMC_DEBUG"):  # finish reports "unknown judge session"
                        traceback.print_exc()
                    if kind in ("sess_open", "sess_extend"):
                        seq = self.sessions.pop(item[1], None)
                        if seq is not None:
                            self.engine.free_sequence(seq)
            # 2. admit waiting requests into free rows (prefilled together)
            if waiting and bat.free_rows and not stop:
                take = [waiting.popleft() for _ in range(min(bat.free_rows, len(waiting)))]
                t0 = time.monotonic_ns()
                seqs, ids_list, reqs = [], [], []
                for kind, req, seq, keep in take:
                    if kind == "gen":
                        seq = self.engine.new_sequence()
                    elif keep < seq.length:  # drop the prefilled tail the full tokenization differs on
                        self.engine.truncate(seq, keep)
                    seqs.append(seq)
                    ids_list.append(req.ids)
                    reqs.append(req)
                try:
                    if stage == "crash":
                        os._exit(17)
                    if stage in ("init", "prefill"):
                        raise InjectedFault(f"injected fault: {self.name} {stage}")
                    self.engine.prefill(seqs, ids_list)
                except Exception as e:  # noqa: BLE001
                    for seq, req in zip(seqs, reqs):
                        self.engine.free_sequence(seq)
                        fail(req, e)
                    seqs = []
                for seq, req, ids in zip(seqs, reqs, ids_list):
                    try:
                        bat.admit(seq, SamplingParams(**req.params), tag=[req, t0, 0, len(ids)], ctx=req.ctx)
                    except Exception as e:  # noqa: BLE001
                        self.engine.free_sequence(seq)
                        fail(req, e)
            # 3. one replay for every live row; report the rows it retired
            if bat.rows:
                try:
                    gone = bat.step()
                except Exception as e:  # noqa: BLE001 - engine failure: every live request fails
                    gone = list(bat.rows)
                    bat.rows = []
                    for row in gone:
                        row.error = row.error or e
                for row in gone:
                    req, t0, ttft, plen = row.tag
                    if row.error is not None:
                        fail(req, row.error)
                    else:
                        self._emit("done", req.rid, {"prompt_tokens": plen, "output_tokens": len(row.tokens),
                                                     "ttft_ns": ttft, "latency_ns": time.monotonic_ns() - t0})
                        if self.on_finished is not None:
                            self.on_finished(req.rid)
                    sent.pop(req.rid, None)
                    self.engine.free_sequence(row.seq)

    def _generate(self, batch: List[_Req], SP) -> None:
        seqs = [self.engine.new_sequence() for _ in batch]
        try:
            self._run(seqs, batch, [r.ids for r in batch], SP)
        finally:
            for s in seqs:
                self.engine.free_sequence(s)

    def _run(self, seqs, reqs: List[_Req], prompts, SP) -> None:
        from ..context import Context

        t0 = time.monotonic_ns()
        stage, k = self.fault or ("", 0)
        if stage == "crash":
            os._exit(17)  # simulated worker death (no cleanup, like a segfault or OOM kill)
        if stage in ("init", "prefill"):
            raise InjectedFault(f"injected fault: {self.name} {stage}")
        self.engine.prefill(seqs, prompts)
        params = [SP(**r.params) for r in reqs]
        first = [0] * len(reqs)
        sent = [0] * len(reqs)

        def on_tokens(i, ids):
            if not first[i]:
                first[i] = time.monotonic_ns() - t0
            if stage == "decode" and sent[i] + len(ids) >= k:
                raise InjectedFault(f"injected fault: {self.name} decode after {k} tokens")
            sent[i] += len(ids)
            self._emit("tokens", reqs[i].rid, ids)

        # a batch is cancelled only if every member is; single requests use their own context
        ctx = reqs[0].ctx if len(reqs) == 1 else _AllCtx([r.ctx for r in reqs])
        del Context
        outs = self.engine.decode(seqs, params, ctx, on_tokens)
        t1 = time.monotonic_ns()
        for i, r in enumerate(reqs):
            self._emit("done", r.rid, {"prompt_tokens": len(prompts[i]), "output_tokens": len(outs[i]),
                                       "ttft_ns": first[i], "latency_ns": t1 - t0})


class _AllCtx:
    """Context view over a batch: done only when every member is cancelled."""

    def __init__(self, ctxs):
        self.ctxs = ctxs

    def done(self) -> bool:
        return all(c.done() for c in self.ctxs)

    def err(self):
        return self.ctxs[0].err()

    def check(self) -> None:
        if self.done():
            from ..context import ContextError

            raise ContextError(self.err())


def worker_main(gpu: int, conn, models: List[dict], dist_info: Optional[dict], trace_on: bool) -> None:
    """Entry point of a worker process (multiprocessing spawn target)."""
    # The driver owns stdout (--json writes the result there); native libraries in the worker
    # (gloo's connection banner, RCCL debug output) print to fd 1 -> send it to stderr.
    try:
        import sys

        sys.stdout.flush()
        os.dup2(2, 1)
    except OSError:
        pass
    send_lock = threading.Lock()

    def send(msg) -> None:
        with send_lock:
            conn.send(msg)

    try:
        from ..utils import trace

        trace.enable(trace_on)
        with trace.span("worker_import", cat="startup", gpu=gpu):
            import torch

            from ..context import Context
            from .. import ops
            from ..engine import Engine, EngineConfig
            from ..models.config import FAMILIES
            from ..parallel.comm import TPGroup

        on_cpu = gpu < 0  # CPU worker (tests / no-GPU hosts): oracle op path, gloo collectives
        if not on_cpu:
            with trace.span("device_init", cat="startup", gpu=gpu):
                torch.cuda.set_device(gpu)
                torch.zeros(1, device=f"cuda:{gpu}")  # HIP context + allocator up front
        groups = {}
        if dist_info:
            import torch.distributed as dist

            kw = {} if on_cpu else {"device_id": torch.device("cuda", gpu)}
            dist.init_process_group("gloo" if on_cpu else "nccl", init_method=f"tcp://127.0.0.1:{dist_info['port']}",
                                    rank=dist_info["rank"], world_size=dist_info["world"], **kw)
            for gname, ranks in dist_info["groups"]:  # every worker creates every group, same order
                g = dist.new_group(ranks)
                # host control channel of the TP group (leader decisions, fault agreement)
                ctrl = g if on_cpu else dist.new_group(ranks, backend="gloo", timeout=CTRL_TIMEOUT)
                if dist_info["rank"] in ranks:
                    groups[gname] = (g, ranks.index(dist_info["rank"]), len(ranks), ctrl)
        hosts: Dict[str, _EngineHost] = {}
        ctxs: Dict[int, Context] = {}  # live requests' contexts (cancel); dropped when they finish
        faults = parse_faults(os.environ.get("LLMC_FAULT", ""))
        for m in models:
            cfg = FAMILIES.get(m["family"])
            if cfg is None and m.get("checkpoint"):  # --weights-dir family (spawned: re-register)
                from ..models.checkpoint import register_dir

                register_dir(m["checkpoint"])
                cfg = FAMILIES[m["family"]]
            if m["name"] in groups:
                g, r, n, ctrl = groups[m["name"]]
                tp = TPGroup(g, r, n, ctrl=ctrl)
                if not on_cpu and os.environ.get("LLMC_CUSTOM_AR", "1") != "0":
                    tp.enable_custom(f"cuda:{gpu}")  # collective over the group: same order on every rank
            else:
                tp = TPGroup.single()
            # TP decode is graph-captured: over the custom xGMI kernels, or — for a group whose peers
            # could not be mapped — over RCCL if the group's capture self-check passes on every rank
            # (collective, same order on every rank); eager only if that fails too
            graphs = tp.size == 1 or tp.custom is not None or (not on_cpu and tp.graph_capture_ok(f"cuda:{gpu}"))
            ecfg = EngineConfig(device="cpu" if on_cpu else f"cuda:{gpu}", max_context=m["max_context"],
                                max_batch=m.get("max_batch", 1), max_seqs=m.get("max_seqs", 0), seed=m["seed"],
                                kv_blocks=m.get("kv_blocks", 0),
                                use_graphs=graphs,
                                # the placement's rule (placement.fused_ar_plan): no fused
                                # all-reduce beside an engine that decodes at the same time
                                fused_ar=bool(m.get("fused_ar", True)),
                                # placement.alone_plan: the lone-engine fused attention + o_proj
                                attn_oproj_min_chunk=ops.attn_oproj_min_chunk(bool(m.get("alone", False))),
                                # MoE under TP: whole experts per rank (LLMC_EXPERT_PARALLEL=1)
                                expert_parallel=os.environ.get("LLMC_EXPERT_PARALLEL", "0") == "1")
            with trace.span("engine_init", cat="startup", engine=m["name"]):
                eng = Engine(cfg, ecfg, tp=tp, name=m["name"])
            hosts[m["name"]] = _EngineHost(m["name"], eng, send, tp.is_leader, faults.get(m["name"]),
                                           on_finished=lambda rid: ctxs.pop(rid, None))
        if not on_cpu:
            # capture all decode graphs now, while nothing else runs in this process
            for h in hosts.values():
                with trace.span("graph_warmup", engine=h.name):
                    h.engine.warmup_graphs()
            torch.cuda.synchronize()
        send(("ready", {"gpu": gpu, "models": list(hosts)}))
    except Exception as e:  # noqa: BLE001
        send(("fatal", f"worker gpu{gpu} init failed: {type(e).__name__}: {e}\n{traceback.format_exc()}"))
        return

    sess_host: Dict[int, _EngineHost] = {}
    while True:
        try:
            msg = conn.recv()
        except EOFError:
            break
        kind = msg[0]
        if kind == "shutdown":
            break
        if kind == "generate":
            _, rid, model, ids, params = msg
            ctx = Context.background()
            ctxs[rid] = ctx
            hosts[model].q.put(("gen", _Req(rid, ids, params, ctx)))
        elif kind == "cancel":
            c = ctxs.get(msg[1])
            if c is not None:
                c.cancel()
        elif kind == "sess_open":
            _, sid, model, ids = msg
            sess_host[sid] = hosts[model]
            hosts[model].q.put(("sess_open", sid, ids))
        elif kind == "sess_extend":
            _, sid, ids = msg
            if sid in sess_host:
                sess_host[sid].q.put(("sess_extend", sid, ids))
        elif kind == "sess_generate":
            _, sid, rid, ids, params, keep = msg
            ctx = Context.background()
            ctxs[rid] = ctx
            sess_host.pop(sid).q.put(("sess_generate", sid, _Req(rid, ids, params, ctx), keep))
        elif kind == "sess_close":
            h = sess_host.pop(msg[1], None)
            if h is not None:
                h.q.put(("sess_close", msg[1]))
        elif kind == "trace":
            from ..utils import trace

            send(("trace", trace.drain()))
    for h in hosts.values():
        h.q.put(None)
    for h in hosts.values():
        h.t.join(timeout=30)
    try:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        pass
