"""Continuous batching over one engine's decode rows (the serving path).

``Engine.decode`` runs a fixed set of rows until every one finishes: a request that arrives while
a batch decodes waits for the whole batch. Here rows join and leave between HIP-graph replays:

* ``admit`` binds a prefilled sequence to the next free row (rows stay compact, 0..B-1, so the
  graph captured for B rows serves them): block table, sampling parameters and the first token
  sampled from the row's prefill logits by the sampler kernel on that row alone (a one-row view
  of every state tensor), which also advances the row's device state;
* ``step`` replays the (B rows, attention bucket) graph — S decode steps for every row — then
  consumes the previous replay's pinned token snapshot (one replay behind, as ``Engine.decode``
  does) and retires finished rows: the rows behind them move down (device row copies on the
  engine stream, ordered after the replay that is still running), so B shrinks.

Every device operation is on the engine's stream, so a retired sequence's KV blocks can be
reused at once: anything that touches them later is ordered after the replays that used them.
TP engines keep ``Engine.decode`` (every rank would have to admit rows at the same replay).
"""

from __future__ import annotations

from typing import Callable, List, Optional

import torch

from .. import ops
from .engine import Engine, EngineError, SamplingParams, Sequence

TokenFn = Callable[["Row", List[int]], None]


class Row:
    __slots__ = ("seq", "params", "tag", "produced", "issued", "base", "done", "error", "ctx", "tokens")

    def __init__(self, seq: Sequence, params: SamplingParams, tag, ctx):
        self.seq = seq
        self.params = params
        self.tag = tag
        self.ctx = ctx
        self.produced = 0   # tokens consumed (streamed) so far
        self.issued = 1     # decode steps issued (the first token comes from the prefill logits)
        self.base = seq.length
        self.done = False
        self.error: Optional[BaseException] = None
        self.tokens: List[int] = []


class ContinuousBatcher:
    def __init__(self, engine: Engine, on_tokens: Optional[TokenFn] = None):
        if engine.tp.size != 1:
            raise EngineError("continuous batching needs a TP=1 engine")
        self.e = engine
        self.on_tokens = on_tokens
        self.rows: List[Row] = []
        self._pending = None          # event of the in-flight host snapshot
        self._snap: List[Row] = []    # row layout the snapshot was taken with
        # host copy of the engine's decode-attention fault word, taken with every snapshot
        self._host_fault = (torch.zeros(1, dtype=torch.int32, pin_memory=True) if engine.on_gpu
                            else torch.zeros(1, dtype=torch.int32))
        self._eos = set(engine.cfg.eos)
        e = engine
        self._row_state = [e.tokens_in, e.positions, e.seq_lens, e.slots, e.block_tables, e.out_tokens,
                           e.out_count, e.next_tok, e.inv_temp, e.top_k, e.top_p, e.seeds]

    @property
    def free_rows(self) -> int:
        return self.e.ecfg.max_batch - len(self.rows)

    # -- admission ------------------------------------------------------------------------------
    @torch.no_grad()
    def admit(self, seq: Sequence, params: SamplingParams, tag=None, ctx=None) -> Row:
        e = self.e
        S = e.ecfg.steps_per_graph
        if not self.free_rows:
            raise EngineError("no free decode row")
        if not seq.has_logits:
            raise EngineError("sequence has no prefill logits")
        if params.max_tokens > e.cap - 2 * S - 1:
            raise EngineError("max_tokens exceeds engine capacity")
        # a row runs at most one replay past its last consumed token before it is retired
        e._reserve(seq, seq.length + params.max_tokens + 2 * S + 1)
        r = len(self.rows)
        with e._on_stream():
            e.block_tables[r:r + 1].copy_(e._block_table([seq]))
            e.logits_local[r].copy_(seq.logits)
            e.inv_temp[r] = 0.0 if params.temperature <= 0 else 1.0 / params.temperature
            e.top_k[r] = params.top_k
            e.top_p[r] = params.top_p
            e.seeds[r] = params.seed
            e.positions[r] = seq.length - 1
            e.out_count[r] = 0
            sl = slice(r, r + 1)
            ops.sample(e.logits_local[sl], e.inv_temp[sl], e.top_k[sl], e.top_p[sl], e.seeds[sl], e.positions[sl],
                       e.next_tok[sl], e.ws_v[sl] if e.ws_v is not None else None,
                       e.ws_i[sl] if e.ws_i is not None else None, tokens_in=e.tokens_in[sl], seq_lens=e.seq_lens[sl],
                       slots=e.slots[sl], block_tables=e.block_tables[sl], bs=e.bs, out_tokens=e.out_tokens[sl],
                       out_count=e.out_count[sl], use_topkp=params.top_k > 0 or params.top_p < 1.0)
        seq.row = r
        row = Row(seq, params, tag, ctx)
        self.rows.append(row)
        return row

    # -- decode ---------------------------------------------------------------------------------
    def _consume(self, counts, toks, layout: List[Row]) -> None:
        for i, row in enumerate(layout):
            if row.done:
                continue
            if row.ctx is not None and row.ctx.done():
                from ..context import ContextError

                row.error, row.done = ContextError(row.ctx.err()), True
                continue
            p = row.params
            n = min(int(counts[i]), p.max_tokens)
            new = toks[i][row.produced:n].tolist() if n > row.produced else []
            stop = False
            if p.stop_on_eos:
                hit = next((j for j, t in enumerate(new) if t in self._eos), -1)
                if hit >= 0:
                    new, stop = new[:hit], True
            if new:
                row.tokens.extend(new)
                if self.on_tokens is not None:
                    try:
                        self.on_tokens(row, new)
                    except Exception as ex:  # noqa: BLE001 - the row's consumer failed: retire it
                        row.error, row.done = ex, True
                        continue
            row.produced = n if not stop else row.produced + len(new)
            if stop or n >= p.max_tokens:
                row.done = True

    def _compact(self) -> List[Row]:
        """Drop finished rows; the live rows behind them move down (device row copies)."""
        keep = [r for r in self.rows if not r.done]
        gone = [r for r in self.rows if r.done]
        if not gone:
            return []
        with self.e._on_stream():
            for t, row in enumerate(keep):
                s = row.seq.row
                if s != t:
                    for buf in self._row_state:
                        buf[t].copy_(buf[s])
                    row.seq.row = t
        self.rows = keep
        for row in gone:
            row.seq.length = row.base + len(row.tokens)
            row.seq.has_logits = False
            row.seq.row = -1
        return gone

    @torch.no_grad()
    def step(self) -> List[Row]:
        """One replay (S tokens for every row that still needs them) + bookkeeping; returns the
        rows retired by this call (``done``; ``error`` set if they failed)."""
        e = self.e
        S = e.ecfg.steps_per_graph
        B = len(self.rows)
        need = any(not r.done and r.issued < r.params.max_tokens for r in self.rows)
        with e._on_stream():
            if need and B:
                bucket = e._bucket(max(r.base + r.issued for r in self.rows) + S + 1)
                e._use_topkp = any(r.params.top_k > 0 or r.params.top_p < 1.0 for r in self.rows)
                graph = e._graph(B, bucket) if (e.on_gpu and e.ecfg.use_graphs) else None
                if graph is not None:
                    graph.replay()
                else:
                    for _ in range(S):
                        e._decode_step(B, bucket)
                for r in self.rows:
                    r.issued += S
            if not e.on_gpu:
                self._consume(e.out_count, e.out_tokens, self.rows)
                return self._compact()
            if self._pending is not None:
                self._pending.synchronize()
                if int(self._host_fault[0]):
                    # a decode-attention merge gave up in the replay behind this snapshot (the
                    # device word is re-armed right after each snapshot's copy, so it covers
                    # exactly that replay, whose rows are all in ``_snap``): fail them instead of
                    # streaming their tokens
                    self._host_fault.zero_()
                    for row in self._snap:
                        if not row.done:
                            row.error, row.done = EngineError("decode attention: a partial merge timed out: "
                                                              "this request's tokens are invalid"), True
                self._consume(e.host_count, e.host_tokens, self._snap)
            gone = self._compact()
            # snapshot of the state after this replay (and the compaction), read next call
            e.host_count.copy_(e.out_count, non_blocking=True)
            e.host_tokens.copy_(e.out_tokens, non_blocking=True)
            self._host_fault.copy_(e.attn_fault, non_blocking=True)
            # re-arm before the next replay is queued: a fault that replay raises lands in the next
            # snapshot instead of being wiped by a clear queued behind it
            e.attn_fault.zero_()
            ev = torch.cuda.Event()
            ev.record(e.stream)
            self._pending, self._snap = ev, list(self.rows)
        return gone

    def drain(self) -> List[Row]:
        """Step until every row is retired."""
        out: List[Row] = []
        while self.rows:
            out.extend(self.step())
        return out
