"""Inference engine: paged-KV prefill + HIP-graph decode for one model instance (T2).

One ``Engine`` = one model replica (or one TP shard of it) on one GPU, with its own hipStream, KV
pool and captured decode graphs; several engines can share a GPU (responders + judge) and run
concurrently on their streams.

Decode is device-resident: tokens, positions, slots, seq_lens, sampling params and the token
history live in device buffers; one decode step = embedding → L × (qkv GEMV [fused RMSNorm] →
RoPE + paged-KV write → split-KV attention → o GEMV [+residual] → gate_up GEMV [fused RMSNorm,
SiLU·up epilogue] → down GEMV [+residual]) → lm_head GEMV [fused final norm] → sample + advance.
``steps_per_graph`` such steps are captured into ONE HIP graph and replayed; the host only polls
the token history (pinned async copy + event, one replay behind) for streaming, EOS, deadline
and cancellation — there is no per-token host↔device synchronisation.

Prefill is eager, chunked (``prefill_chunk`` tokens), on MFMA GEMMs + the flash prefill kernel
over the paged cache; a prefill may extend an existing sequence (incremental judge prefill,
SURVEY.md §7.4).
"""

from __future__ import annotations

import dataclasses
import math
import os
import time
from typing import Callable, Dict, List, Optional, Sequence as Seq

import torch

from .. import ops
from ..context import Context, ContextError
from ..models.config import ModelConfig, rope_inv_freq
from ..models.transformer import TransformerWeights
from ..ops import EPI_BF16, EPI_F32, EPI_RESADD, EPI_SILU, oracle
from ..parallel.comm import TPGroup
from ..utils import trace
from ..utils.native import runtime


@dataclasses.dataclass
class EngineConfig:
    device: str = "cuda:0"
    max_context: int = 8192
    max_batch: int = 1   # decode rows per step (weight-streaming GEMV/MFMA form: M <= 32; MoE <= 16)
    max_seqs: int = 0    # live sequences the KV pool is sized for (0 = max_batch)
    block_size: int = 64
    kv_blocks: int = 0
    seed: int = 0
    steps_per_graph: int = 8
    use_graphs: bool = True
    prefill_chunk: int = 8192
    init_scale: float = 1.0
    stream_priority: int = 0
    # rehearsals only: run this engine's stream on CUs [lo, hi] ("lo-hi"; default LLMC_CU_MASK), so
    # TP ranks sharing one GPU each get CUs of their own, as they would have GPUs of their own
    cu_mask: str = dataclasses.field(default_factory=lambda: os.environ.get("LLMC_CU_MASK", ""))
    # TP prefill: shard the residual stream by token rows between layers (reduce-scatter +
    # all-gather instead of all-reduce) for chunks of >= sp_min_tokens tokens
    sequence_parallel: bool = True
    sp_min_tokens: int = 256
    # MoE under TP: each rank holds n_experts / tp whole experts instead of 1/tp of every expert
    expert_parallel: bool = False
    # one-row engines without TP: decode attention + o_proj + residual as ONE launch per layer
    # (csrc/kernels/attn_oproj.hip) in the context buckets with at least ``attn_oproj_min_chunk``
    # keys per block (ops.ATTN_OPROJ_MIN_CHUNK: where it measured faster than the two launches).
    # Environment defaults (A/B runs): LLMC_ATTN_OPROJ=0 never, =all every bucket it covers.
    attn_oproj: bool = dataclasses.field(default_factory=lambda: os.environ.get("LLMC_ATTN_OPROJ", "1") != "0")
    # tensor-parallel ranks too: the rank's o_proj share as the launch's partial, its all-reduce in
    # the kernel's tile-reducer epilogue when the group has the fused buffer (``fused_ar``), else the
    # separate all-reduce launch after it (LLMC_TP_ATTN_OPROJ=0: the two launches, A/B runs)
    # Measured slower on every 8B TP shape (MI355X, 2k keys, rank alone: TP=8 0.876 -> 1.047 ms/token,
    # TP=4 1.143 -> 1.326; 2-rank TP=8-shaped rehearsal with collectives 1.356 -> 1.474): a rank's
    # 1-4 kv heads make the head merge the long pole and the o_proj it hides is small, so the
    # default keeps the one-launch qkv + attention and the o GEMV with its fused all-reduce
    # (LLMC_TP_ATTN_OPROJ=1: A/B runs; profiles/r6_tp_decode.md)
    tp_attn_oproj: bool = dataclasses.field(default_factory=lambda: os.environ.get("LLMC_TP_ATTN_OPROJ", "0") == "1")
    attn_oproj_min_chunk: int = dataclasses.field(default_factory=ops.attn_oproj_min_chunk)
    # one-row engines: the qkv projection and the decode attention as ONE launch in the buckets of
    # the fused attention form (csrc/kernels/qkv_attn.hip). "1": shards whose qkv output is under
    # QKV_ATTN_MAX_ROWS rows (the TP ranks', where it measured faster: profiles/r4_qkv_attn.md);
    # "all": every covered shape and fused bucket, ahead of attn_oproj; "0": never (LLMC_QKV_ATTN)
    qkv_attn: str = dataclasses.field(default_factory=lambda: os.environ.get("LLMC_QKV_ATTN", "1"))
    # ... and the token's o_proj (+ the TP all-reduce in its epilogue, ``fused_ar``) in the same
    # launch (the o-role of csrc/kernels/qkv_attn.hip) instead of the o GEMV after it (LLMC_QKV_ATTN_O)
    qkv_attn_o: bool = dataclasses.field(default_factory=lambda: os.environ.get("LLMC_QKV_ATTN_O", "0") == "1")
    # MoE engines alone on one GPU: in the buckets that run the fused attention + o_proj's whole-row
    # form, the decode router (RMSNorm -> logits -> top-k) inside that launch instead of its own
    # launch after it (csrc/kernels/attn_oproj.hip AoRouter; LLMC_AO_ROUTER=0: the router launch)
    ao_router: bool = dataclasses.field(default_factory=lambda: os.environ.get("LLMC_AO_ROUTER", "1") != "0")
    # TP engines: the decode all-reduce inside the row-parallel GEMVs' epilogue when the group has
    # the fused buffer (TPGroup.custom_fused). Its 256 blocks spin per block on their peers, so an
    # engine whose GPUs also run other engines' decode at the same time (bench.py's N=2 third
    # responder) keeps the separate, 64-block all-reduce launch
    fused_ar: bool = True


FUSED_CHUNK_SMALL, FUSED_CHUNK_LARGE = 128, 256
# one-launch qkv + attention by default only for qkv outputs under this many rows (TP shards)
QKV_ATTN_MAX_ROWS = 2048
# batching engines: minimum keys per split block (see attn_buckets) when rows x kv heads fill the
# chip with >= 32 (row, head) units, and below that (3 duplicate 8B responders = 24 units, TP
# ranks holding 1-2 kv heads) where a row needs more blocks of its own
BATCHING_MIN_KEYS, BATCHING_MIN_KEYS_FEW = 2048, 512


def attn_buckets(ctxmax: int, blocks_per_head: int = 32, fused_max: int = 4096, group: int = 4,
                 nkv: int = 8, rows: int = 1) -> List[tuple]:
    """Decode-attention shapes per context bucket: [(capacity_tokens, chunk, grid_chunks, fused)].

    Capacities double from 1024. A bucket uses the fused form (fixed-chunk blocks over the bucket
    capacity, grid_chunks = capacity / chunk; no length-dependent page-table round trip) up to
    ``fused_max`` keys — 128-key chunks up to 2048 keys with GQA (``group`` query heads per kv
    head >= 2) and up to 1024 without (Phi-3), 256-key chunks above — and, beyond it, while the
    grid stays within ~one block per CU: 128-key chunks if capacity / 128 x ``nkv`` <= 256, else
    256-key chunks if capacity / 256 x ``nkv`` <= 256 (TP ranks, whose one or two kv heads leave
    the chip idle under a per-head split). Otherwise the balanced split: ``chunk`` is the minimum
    of 128 keys per block, the kernel spreads a sequence's keys evenly over ``grid_chunks`` blocks,
    and the grid grows with the context until ``blocks_per_head``; one bucket then covers every
    longer context. Measured per shape: profiles/r2_attn_decode.md. ``fused_max`` = 0 disables
    the fused form (page size not a multiple of 32 keys).

    An engine batching ``rows`` >= 3 decode rows uses the balanced split with a minimum of ``mk``
    keys per block over min(32, capacity / mk) blocks per kv head — mk = BATCHING_MIN_KEYS (2048)
    when rows x kv heads give >= 32 independent (row, head) units, BATCHING_MIN_KEYS_FEW (512)
    below — always on 8-wave blocks: a row of L keys is split into min(32, ceil(L / mk)) ranges
    whatever the bucket and whatever else is batched, so its tokens are batch-invariant (the fused
    form's chunk and the split grid would follow the bucket the longest row selects); a lone long
    row still spreads over the chip (8B at 13.5k keys: 30 µs vs 141 for one block per (row,
    head)) while 32 rows stay within 1.2x of it (profiles/r2_batched_decode.md,
    `microbench_kernels.py attn-rows`)."""
    out, cap = [], 1024
    if rows >= 3:
        mk = BATCHING_MIN_KEYS if rows * nkv >= 32 else BATCHING_MIN_KEYS_FEW
        while True:
            c = min(cap, ctxmax)
            gc = min(32, (c + mk - 1) // mk)
            if out and out[-1][2] == gc:
                out[-1] = (c, mk, gc, False)
            else:
                out.append((c, mk, gc, False))
            if cap >= ctxmax:
                return out
            cap *= 2
    while True:
        c = min(cap, ctxmax)
        if fused_max > 0 and c <= fused_max:
            ch = FUSED_CHUNK_SMALL if c <= (2048 if group >= 2 else 1024) else FUSED_CHUNK_LARGE
            out.append((c, ch, (c + ch - 1) // ch, True))
        elif fused_max > 0 and (c + 127) // 128 * nkv <= 256:
            out.append((c, 128, (c + 127) // 128, True))
        elif fused_max > 0 and (c + 255) // 256 * nkv <= 256:
            out.append((c, 256, (c + 255) // 256, True))
        else:
            gc = min((c + 127) // 128, blocks_per_head)
            if out and not out[-1][3] and out[-1][2] == gc:
                out[-1] = (c, 128, gc, False)  # same grid: widen the previous bucket
            else:
                out.append((c, 128, gc, False))
        if cap >= ctxmax:
            return out
        cap *= 2


def qkv_attn_plan(buckets: List[tuple], ao_chunks: List[int], mode: str, qkv_rows: int, bs: int):
    """Per decode-attention bucket the (keys per block, blocks per kv head) of the one-launch qkv +
    attention (csrc/kernels/qkv_attn.hip) or None, and the attn_oproj chunks it leaves, for a one-row
    engine whose shape the kernel covers. ``mode`` (EngineConfig.qkv_attn): "0" never; "1" the
    fused-form buckets of shards with fewer than QKV_ATTN_MAX_ROWS qkv rows where attn_oproj does not
    run (the TP ranks: profiles/r4_qkv_attn.md); "all" every bucket, ahead of attn_oproj, the split-form
    ones as 256-key blocks (measured slower on wide outputs; A/B runs)."""
    plan: List[Optional[tuple]] = [None] * len(buckets)
    if mode in ("0", "False", "") or (mode != "all" and qkv_rows >= QKV_ATTN_MAX_ROWS):
        return plan, list(ao_chunks)
    qa_all = mode == "all"
    for i, (cap, ch, gc, fused) in enumerate(buckets):
        if fused and ch in (128, 256) and bs % (ch // 4) == 0 and (qa_all or not ao_chunks[i]):
            plan[i] = (ch, gc)
        elif qa_all and not fused and bs % 64 == 0:
            plan[i] = (256, (cap + 255) // 256)
    ao = [0 if q else a for q, a in zip(plan, ao_chunks)] if qa_all else list(ao_chunks)
    return plan, ao


def split_blocks_per_head(nh: int, nkv: int) -> int:
    """Grid of the split (long-context) attention form per kv head: ~one block per CU over the row's
    kv heads (256; 512 without GQA, where a block's range costs less). A TP=8 rank's single kv
    head gets all 256 (its partials merge in two levels of 16)."""
    blocks = 512 if nh == nkv else 256
    return max(1, min(blocks // nkv, 256))


@dataclasses.dataclass
class SamplingParams:
    max_tokens: int = 256
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    seed: int = 0
    stop_on_eos: bool = True


class Sequence:
    """A KV-cache-backed token sequence. It is bound to a decode row only while it decodes."""

    def __init__(self, sid: int):
        self.sid = sid
        self.row = -1
        self.blocks: List[int] = []
        self.length = 0
        self.has_logits = False
        self.logits: Optional[torch.Tensor] = None  # last-token logits [V_local] after prefill


class EngineError(Exception):
    pass


class InjectedEngineFault(EngineError):
    """Raised by the ``Engine.fault_at`` test hook."""


class _TPBroken(EngineError):
    """The TP group of this engine can no longer agree (see Engine._tp_broken)."""


class Engine:
    def __init__(self, cfg: ModelConfig, ecfg: Optional[EngineConfig] = None, tp: Optional[TPGroup] = None,
                 name: str = "", weights: Optional[TransformerWeights] = None):
        self.cfg = cfg
        self.ecfg = ecfg or EngineConfig()
        rows_max = ops.MOE_GEMVM_MAX_TOKENS if cfg.is_moe else ops.GEMV_MAX_M
        if not 1 <= self.ecfg.max_batch <= rows_max:
            raise EngineError(f"{cfg.name}: max_batch {self.ecfg.max_batch} outside 1..{rows_max} decode rows")
        self.tp = tp or TPGroup.single()
        self.name = name or cfg.name
        self.device = torch.device(self.ecfg.device)
        self.on_gpu = self.device.type == "cuda"
        # decode projections of an engine that batches >= 3 rows run on the MFMA form at every row
        # count (ops.linear ``mfma``): one numeric form per engine, so a request's tokens do not
        # depend on how many rows shared its steps; 1-2 row engines keep the faster VALU GEMV
        self.mfma_decode = self.on_gpu and self.ecfg.max_batch >= 3
        if self.on_gpu:
            torch.cuda.set_device(self.device)
            if self.ecfg.cu_mask:
                lo, hi = (int(v) for v in self.ecfg.cu_mask.split("-"))
                words = [0] * max(8, hi // 32 + 1)
                for cu in range(lo, hi + 1):
                    words[cu // 32] |= 1 << (cu % 32)
                from ..utils.native import kernels

                ptr = kernels().stream_cu_mask(self.device.index or 0, words)
                self.stream = torch.cuda.ExternalStream(ptr, device=self.device)
            else:
                self.stream = torch.cuda.Stream(self.device, priority=self.ecfg.stream_priority)
        else:
            self.stream = None
        e = self.ecfg
        with self._on_stream():
            with trace.span("weights_init", engine=self.name):
                if weights is not None:
                    self.w = weights.to(self.device)
                else:
                    self.w = TransformerWeights(cfg, self.tp, self.device, e.seed, e.init_scale,
                                                expert_parallel=e.expert_parallel)
        self.nh, self.nkv, self.D = self.w.nh, self.w.nkv, cfg.head_dim
        self.scale = 1.0 / math.sqrt(self.D)
        self.bs = e.block_size
        self.max_blocks_per_seq = (e.max_context + self.bs - 1) // self.bs + 1
        nb = e.kv_blocks or max(e.max_seqs, e.max_batch) * self.max_blocks_per_seq + 2
        self.alloc = runtime().BlockAllocator(nb, self.bs)
        dev = self.device
        L = cfg.n_layers
        self.k_cache = torch.zeros(L, nb, self.nkv, self.bs, self.D, dtype=torch.bfloat16, device=dev)
        self.v_cache = torch.zeros_like(self.k_cache)
        cos_t, sin_t = oracle.rope_tables(rope_inv_freq(cfg), e.max_context + e.steps_per_graph + 2)
        self.cos_t, self.sin_t = cos_t.to(dev), sin_t.to(dev)
        self._alloc_decode_buffers()
        self._graphs: Dict[int, "torch.cuda.CUDAGraph"] = {}
        self._next_sid = 0

    # ------------------------------------------------------------------------------------------
    def _on_stream(self):
        if self.stream is not None:
            return torch.cuda.stream(self.stream)
        import contextlib

        return contextlib.nullcontext()

    def _alloc_decode_buffers(self) -> None:
        B, dev, c = self.ecfg.max_batch, self.device, self.cfg
        i32 = dict(dtype=torch.int32, device=dev)
        self.tokens_in = torch.zeros(B, **i32)
        self.positions = torch.zeros(B, **i32)
        self.seq_lens = torch.ones(B, **i32)
        self.slots = torch.zeros(B, **i32)
        self.block_tables = torch.zeros(B, self.max_blocks_per_seq, **i32)
        self.cap = self.ecfg.max_context + self.ecfg.steps_per_graph + 1
        self.out_tokens = torch.zeros(B, self.cap, **i32)
        self.out_count = torch.zeros(B, **i32)
        self.next_tok = torch.zeros(B, **i32)
        self.inv_temp = torch.ones(B, dtype=torch.float32, device=dev)
        self.top_k = torch.zeros(B, **i32)
        self.top_p = torch.ones(B, dtype=torch.float32, device=dev)
        self.seeds = torch.zeros(B, dtype=torch.int64, device=dev)
        bf = dict(dtype=torch.bfloat16, device=dev)
        self.h = torch.zeros(B, c.hidden, **bf)
        self.q = torch.zeros(B, self.w.q_size, **bf)
        self.attn = torch.zeros(B, self.w.q_size, **bf)
        self.act = torch.zeros(B, self.w.inter, **bf)
        self.logits_local = torch.zeros(B, self.w.vocab_local, dtype=torch.float32, device=dev)
        self.logits = (self.logits_local if self.tp.size == 1
                       else torch.zeros(B, c.vocab, dtype=torch.float32, device=dev))
        self._gather_buf = (None if self.tp.size == 1 else
                            torch.zeros(self.tp.size, B, self.w.vocab_local, dtype=torch.float32, device=dev))
        # split-KV decode attention: one (chunk, grid) shape per context bucket
        ctxmax = self.ecfg.max_context + self.ecfg.steps_per_graph + 2
        self.attn_buckets = attn_buckets(ctxmax, split_blocks_per_head(self.nh, self.nkv),
                                         ops.FUSED_ATTN_MAX_KEYS if self.bs % 32 == 0 else 0, self.nh // self.nkv,
                                         self.nkv, rows=self.ecfg.max_batch)
        # fused attention + o_proj launch: per bucket its keys per block (0 = the bucket keeps the
        # two launches)
        self.ao_chunks: List[int] = [0] * len(self.attn_buckets)
        self.ao_nc = 0
        if (self.on_gpu and self.ecfg.attn_oproj and B == 1 and self.bs % 32 == 0
                and (self.tp.size == 1 or self.ecfg.tp_attn_oproj)):
            self.ao_nc = ops.attn_oproj_grid(c.hidden, self.nh, self.nkv, self.D)
            if self.ao_nc:
                lo = self.ecfg.attn_oproj_min_chunk
                # a block of > 256 keys gives each wave two 32-key sub-tiles of one 64-key unit:
                # pages must hold whole units there (the kernel rejects bs % 64 != 0)
                self.ao_chunks = [ch if ch >= lo and (ch <= 256 or self.bs % 64 == 0) else 0
                                  for ch in (ops.attn_oproj_chunk(cap, self.ao_nc) for cap, _, _, _ in self.attn_buckets)]
                self.ao_ws = ops.attn_oproj_workspace(c.hidden, self.nh, self.nkv, self.D, self.ao_nc, dev)
        # one-launch qkv + attention: per bucket its (chunk, grid) of the fused attention form, or
        # None (B = max_batch: one-row engines only, so a row's tokens never depend on what shared
        # their steps). Default: the fused-form buckets of short-qkv shards where attn_oproj does not
        # run; "all": every bucket, ahead of attn_oproj, the long ones as 256-key chunks
        self.qa_plan: List[Optional[tuple]] = [None] * len(self.attn_buckets)
        if self.on_gpu and B == 1 and ops.qkv_attn_supported(self.nh, self.nkv, self.D, c.hidden):
            self.qa_plan, self.ao_chunks = qkv_attn_plan(self.attn_buckets, self.ao_chunks, str(self.ecfg.qkv_attn),
                                                         (self.nh + 2 * self.nkv) * self.D, self.bs)
            if any(self.qa_plan):
                self.qa_ws = ops.qkv_attn_workspace(self.nh, self.nkv, self.D, dev)
        self.qa_buckets = [p is not None for p in self.qa_plan]
        # MoE router inside the fused attention + o_proj launch (whole-row form buckets)
        self.ao_router = [False] * len(self.attn_buckets)
        if (self.ao_nc and c.is_moe and self.tp.size == 1 and not self.w.ep and self.ecfg.ao_router
                and c.n_experts <= 8 and not self.mfma_decode):
            self.ao_router = [bool(ch) and ops.attn_oproj_form(c.hidden, self.nh, self.nkv, self.D, self.ao_nc, ch) == 2
                              for ch in self.ao_chunks]
            if any(self.ao_router):
                self.ao_rws = ops.attn_oproj_router_workspace(self.nkv, self.ao_nc, dev)
        self.qa_o = (any(self.qa_plan) and self.ecfg.qkv_attn_o
                     and ops.qkv_attn_o_supported(self.nh, self.D, c.hidden))
        max_chunks = max([gc for _, _, gc, _ in self.attn_buckets] + [p[1] for p in self.qa_plan if p])
        self.attn_part, self.attn_counters = ops.decode_attn_workspace(B, self.nh, self.nkv, self.D, max_chunks, dev)
        # set by a decode-attention merger that gave up on a partial (checked after every decode)
        self.attn_fault = torch.zeros(1, dtype=torch.int32, device=dev) if self.on_gpu else None
        if self.on_gpu:
            P = ops.sample_parts()
            self.ws_v = torch.zeros(B, P, dtype=torch.float32, device=dev)
            self.ws_i = torch.zeros(B, P, dtype=torch.int32, device=dev)
        else:
            self.ws_v = self.ws_i = None
        if c.is_moe:
            k = c.top_k_experts
            self.xn = torch.zeros(B, c.hidden, **bf)
            self.router_logits = torch.zeros(B, c.n_experts, dtype=torch.float32, device=dev)
            self.moe_w = torch.zeros(B, k, dtype=torch.float32, device=dev)
            self.moe_ids = torch.zeros(B, k, **i32)
            self.moe_act = torch.zeros(B * k, self.w.inter, **bf)
            self.moe_y = torch.zeros(B * k, c.hidden, **bf)
            self.moe_lw = torch.zeros(B, k, dtype=torch.float32, device=dev)
            self.moe_lids = torch.zeros(B, k, **i32)
        if self.on_gpu:
            self.host_tokens = torch.zeros(B, self.cap, dtype=torch.int32, pin_memory=True)
            self.host_count = torch.zeros(B, dtype=torch.int32, pin_memory=True)

    # -- sequence management -------------------------------------------------------------------
    def new_sequence(self) -> Sequence:
        self._next_sid += 1
        return Sequence(self._next_sid)

    def free_sequence(self, seq: Sequence) -> None:
        if seq.blocks:
            self.alloc.free(seq.blocks)
            seq.blocks = []
        seq.length = 0
        seq.logits = None
        seq.has_logits = False

    def truncate(self, seq: Sequence, length: int) -> None:
        """Forget every token of ``seq`` from position ``length`` on (their KV slots are simply
        overwritten by the next prefill; blocks stay reserved)."""
        if not 0 <= length <= seq.length:
            raise EngineError(f"truncate to {length} of a {seq.length}-token sequence")
        seq.length = length
        seq.logits = None
        seq.has_logits = False

    def _reserve(self, seq: Sequence, total_tokens: int) -> None:
        need = self.alloc.blocks_for(total_tokens) - len(seq.blocks)
        if total_tokens > self.max_blocks_per_seq * self.bs:
            raise EngineError(f"context {total_tokens} exceeds engine max_context {self.ecfg.max_context}")
        if need > 0:
            got = self.alloc.allocate(need)
            if not got:
                raise EngineError(f"KV cache exhausted ({self.alloc.num_free} blocks free, need {need})")
            seq.blocks.extend(got)

    def _block_table(self, seqs: List[Sequence]) -> torch.Tensor:
        """[len(seqs), max_blocks] int32 block table on the engine device."""
        bt = torch.zeros(len(seqs), self.max_blocks_per_seq, dtype=torch.int32)
        for i, s in enumerate(seqs):
            bt[i, : len(s.blocks)] = torch.tensor(s.blocks, dtype=torch.int32)
        return bt.to(self.device, non_blocking=True) if self.on_gpu else bt

    # -- prefill ----------------------------------------------------------------------------------
    @torch.no_grad()
    def prefill(self, seqs: List[Sequence], token_lists: List[List[int]], want_logits: bool = True) -> None:
        """Append ``token_lists[i]`` to ``seqs[i]`` (chunked); optionally compute last-token logits."""
        self._check_usable()
        with self._on_stream(), trace.span("prefill", engine=self.name, tokens=sum(len(t) for t in token_lists)):
            pending = [(s, list(t)) for s, t in zip(seqs, token_lists) if t]
            chunk = self.ecfg.prefill_chunk
            while pending:
                batch, rest, budget, finals = [], [], chunk, set()
                for s, t in pending:
                    if budget <= 0:
                        rest.append((s, t))
                        continue
                    take = t[:budget]
                    batch.append((s, take))
                    budget -= len(take)
                    if len(take) < len(t):
                        rest.append((s, t[len(take):]))
                    else:
                        finals.add(s)
                self._prefill_chunk(batch, want_logits, finals)
                pending = rest

    def _prefill_chunk(self, batch, want_logits: bool, finals) -> None:
        dev, c = self.device, self.cfg
        ids, pos, slots, q_start, q_lens, ctx_lens = [], [], [], [], [], []
        for s, toks in batch:
            self._reserve(s, s.length + len(toks))
            q_start.append(len(ids))
            q_lens.append(len(toks))
            for i, t in enumerate(toks):
                p = s.length + i
                ids.append(t)
                pos.append(p)
                slots.append(s.blocks[p // self.bs] * self.bs + p % self.bs)
            s.length += len(toks)
            ctx_lens.append(s.length)
        T = len(ids)
        i32 = dict(dtype=torch.int32)
        ids_d = torch.tensor(ids, **i32).to(dev, non_blocking=True)
        pos_d = torch.tensor(pos, **i32).to(dev, non_blocking=True)
        slots_d = torch.tensor(slots, **i32).to(dev, non_blocking=True)
        qs_d = torch.tensor(q_start, **i32).to(dev, non_blocking=True)
        ql_d = torch.tensor(q_lens, **i32).to(dev, non_blocking=True)
        cl_d = torch.tensor(ctx_lens, **i32).to(dev, non_blocking=True)
        bt = self._block_table([s for s, _ in batch])
        max_qlen = max(q_lens)
        max_ctx = max(ctx_lens)
        ksplit, kmin = (ops.attn_prefill_plan(len(batch), max_qlen, max_ctx, self.nh, self.nkv, D=self.D, bs=self.bs)
                        if ids_d.is_cuda else (1, 1))
        pws = (ops.attn_prefill_workspace(ksplit, T, self.nh, self.D, dev, len(batch), self.nkv, max_qlen)
               if ksplit > 1 else None)

        h = ops.embedding(ids_d, self.w.embed)
        attn = torch.empty(T, self.w.q_size, dtype=torch.bfloat16, device=dev)
        qbuf = torch.empty(T, self.w.q_size, dtype=torch.bfloat16, device=dev)
        sp = self._sp_plan(T)
        if sp is not None:  # sequence parallel: this rank keeps rows [r*Ts, (r+1)*Ts) of the stream
            Ts, gbuf, pbuf = sp
            r0 = self.tp.rank * Ts
            hs = torch.zeros(Ts, c.hidden, dtype=torch.bfloat16, device=dev)
            mine = max(0, min(T, r0 + Ts) - r0)
            if mine:
                hs[:mine].copy_(h[r0:r0 + mine])
            del h
        for li, Lw in enumerate(self.w.layers):
            if sp is not None:
                xn = self._sp_gather(ops.rmsnorm(hs, Lw.ln1, c.rms_eps), gbuf, T)
            else:
                xn = ops.rmsnorm(h, Lw.ln1, c.rms_eps)
            qkv = ops.linear(xn, Lw.w_qkv, EPI_BF16)
            ops.rope_kv_write(qkv, pos_d, self.cos_t, self.sin_t, self.k_cache[li], self.v_cache[li], slots_d,
                              self.nh, self.nkv, self.D, self.bs, qbuf)
            ops.attn_prefill(qbuf, self.k_cache[li], self.v_cache[li], bt, qs_d, ql_d, cl_d, attn, max_qlen,
                             self.nh, self.nkv, self.D, self.bs, self.scale, max_ctx=max_ctx, ksplit=ksplit, kmin=kmin,
                             ws=pws)
            if sp is not None:
                self._sp_row_parallel(lambda out: ops.linear(attn, Lw.w_o, EPI_RESADD, out=out), hs, pbuf, T)
                if c.is_moe and self.w.ep:
                    # expert parallel on token shards: tokens go to their experts' ranks (all-to-all)
                    self._moe_ep_a2a(ops.rmsnorm(hs, Lw.ln2, c.rms_eps), Lw, hs)
                    continue
                xn = self._sp_gather(ops.rmsnorm(hs, Lw.ln2, c.rms_eps), gbuf, T)
                if c.is_moe:
                    self._sp_row_parallel(lambda out: self._moe(xn, Lw, out, reduce=False), hs, pbuf, T)
                else:
                    act = ops.linear(xn, Lw.w_gu, EPI_SILU)
                    self._sp_row_parallel(lambda out: ops.linear(act, Lw.w_down, EPI_RESADD, out=out), hs, pbuf, T)
                continue
            self._row_parallel(attn, Lw.w_o, h)
            xn = ops.rmsnorm(h, Lw.ln2, c.rms_eps)
            if c.is_moe:
                self._moe(xn, Lw, h)
            else:
                act = ops.linear(xn, Lw.w_gu, EPI_SILU)
                self._row_parallel(act, Lw.w_down, h)
        if sp is not None:  # whole stream back on every rank (only the last rows are read below)
            h = self._sp_gather(hs, sp[1], T)
        # last-token logits for every sequence whose final prompt token is in this chunk
        sel = [i for i, (s, _) in enumerate(batch) if want_logits and s in finals]
        for i0 in range(0, len(sel), ops.GEMV_MAX_M):
            part = sel[i0:i0 + ops.GEMV_MAX_M]
            last_d = torch.tensor([q_start[i] + q_lens[i] - 1 for i in part], dtype=torch.int32).to(dev)
            hl = ops.gather_rows(h, last_d, 1)  # K14 last-token gather
            lg = torch.empty(len(part), self.w.vocab_local, dtype=torch.float32, device=dev)
            ops.linear(hl, self.w.lm_head, EPI_F32, out=lg, norm_w=self.w.final_norm, eps=c.rms_eps,
                       mfma=self.mfma_decode)
            for j, i in enumerate(part):
                s = batch[i][0]
                s.logits = lg[j]
                s.has_logits = True

    # -- sequence parallel (TP prefill) ---------------------------------------------------------
    def _sp_plan(self, T: int):
        """(rows per rank, gather buffer, partial buffer) when this chunk runs sequence parallel."""
        n = self.tp.size
        if n == 1 or not self.ecfg.sequence_parallel or T < max(self.ecfg.sp_min_tokens, n):
            return None
        Ts = (T + n - 1) // n
        H = self.cfg.hidden
        gbuf = torch.empty(n * Ts, H, dtype=torch.bfloat16, device=self.device)
        pbuf = torch.empty(n * Ts, H, dtype=torch.bfloat16, device=self.device)
        return Ts, gbuf, pbuf

    def _sp_gather(self, xs: torch.Tensor, gbuf: torch.Tensor, T: int) -> torch.Tensor:
        """All-gather the row shards [Ts, H] of every rank -> the first T rows of [n*Ts, H]."""
        self.tp.all_gather_rows(xs, gbuf.view(self.tp.size, xs.shape[0], xs.shape[1]))
        return gbuf[:T]

    def _sp_row_parallel(self, accumulate, hs: torch.Tensor, pbuf: torch.Tensor, T: int) -> None:
        """hs += (this row block of) sum_r partial_r: every rank seeds the rows it owns with its
        residual shard (zeros elsewhere), ``accumulate(out)`` adds its partial product into the
        first T rows, and a reduce-scatter leaves each rank its own summed rows — the residual
        is folded in exactly once per row, with no separate add."""
        Ts = hs.shape[0]
        r0 = self.tp.rank * Ts
        pbuf.zero_()
        pbuf[r0:r0 + Ts].copy_(hs)
        accumulate(pbuf[:T])
        self.tp.reduce_scatter_rows(pbuf, hs)

    def _row_parallel(self, x: torch.Tensor, W: torch.Tensor, h: torch.Tensor) -> None:
        """h += x @ W^T across the TP group (residual folded into rank 0's partial). Decode rows
        (<= 2, VALU GEMV form) of a group with mapped peers: ONE launch, the all-reduce in the
        GEMV's epilogue (EPI_AR); otherwise the GEMV/GEMM, then the group's all-reduce."""
        car = self.tp.custom_fused if self.ecfg.fused_ar else None
        if car is not None and h.is_cuda and x.shape[0] <= 2 and not self.mfma_decode and h.is_contiguous():
            car.gemv_allreduce(x, W, h)
            return
        ops.linear(x, W, EPI_RESADD if self.tp.rank == 0 else EPI_BF16, out=h, mfma=self.mfma_decode)
        self.tp.all_reduce_(h)

    def _expert_ffn(self, A: torch.Tensor, ids: torch.Tensor, Lw) -> torch.Tensor:
        """y[p] = down_e(silu(gate_up_e(A[p // k]))) for every (row, slot) pair p of ``ids`` [n, k]
        (expert ids index this rank's expert tensors): expert GEMVs for <= 4 rows, else expert
        alignment + the gathered-row grouped MFMA GEMM (K10/K11: the 256 x 256 LDS-DMA pipeline
        once the pairs average >= 256 rows per expert, 128-row tiles below), SiLU fused into the
        gate_up epilogue."""
        c = self.cfg
        n, k = ids.shape
        E_l, I_l, H = Lw.w_gu.shape[0], self.w.inter, c.hidden
        y = torch.empty(n * k, H, dtype=torch.bfloat16, device=A.device)
        if n == 0:
            return y
        if not A.is_cuda:
            for p in range(n * k):
                e = int(ids.view(-1)[p])
                if e < 0:  # another rank's expert / an all-to-all padding slot: never read
                    y[p].zero_()
                    continue
                gu = (A[p // k:p // k + 1].float() @ Lw.w_gu[e].float().t()).to(torch.bfloat16)
                y[p] = (oracle.silu_mul_interleaved(gu).float() @ Lw.w_down[e].float().t()).to(torch.bfloat16)[0]
            return y
        if n <= ops.MOE_GEMV_MAX_M:
            act = torch.empty(n * k, I_l, dtype=torch.bfloat16, device=A.device)
            ops.moe_gemv(A, Lw.w_gu, ids, k, act, 2 * I_l, H, EPI_SILU)
            ops.moe_gemv(act, Lw.w_down, ids, 1, y, H, I_l, EPI_BF16)
            return y
        tile = ops.moe_tile(n * k, E_l)
        mt = ops.moe_max_tiles(n * k, E_l, tile)
        sr = torch.empty(mt * tile, dtype=torch.int32, device=A.device)
        te = torch.empty(mt, dtype=torch.int32, device=A.device)
        tc = torch.empty(1, dtype=torch.int32, device=A.device)
        ops.moe_align(ids, E_l, sr, te, tc, tile=tile)
        # gate_up with the SiLU-mul in its epilogue: the [pairs, 2I] product never reaches memory
        act = torch.empty(n * k, I_l, dtype=torch.bfloat16, device=A.device)
        ops.moe_gemm(A, Lw.w_gu, sr, te, tc, act, 2 * I_l, H, mt, k, epi=EPI_SILU, tile=tile)
        ops.moe_gemm(act, Lw.w_down, sr, te, tc, y, H, I_l, mt, 1, tile=tile)
        return y

    def _route(self, xn: torch.Tensor, Lw):
        """Prefill router (K9): one fused launch (logits, softmax, top-k) where the kernel covers the
        shape, else the router-logits GEMM + the top-k kernel."""
        c = self.cfg
        T, k = xn.shape[0], c.top_k_experts
        w = torch.empty(T, k, dtype=torch.float32, device=xn.device)
        ids = torch.empty(T, k, dtype=torch.int32, device=xn.device)
        if xn.is_cuda and xn.is_contiguous() and ops.moe_route_fused_supported(c.n_experts, c.hidden):
            ops.moe_route_fused(xn, Lw.w_router, k, w, ids)
            return w, ids
        rl = ops.linear(xn, Lw.w_router, EPI_F32)
        ops.moe_route(rl, k, w, ids)
        return w, ids

    def _moe(self, xn: torch.Tensor, Lw, h: torch.Tensor, reduce: bool = True) -> None:
        """h += MoE(xn). ``reduce`` (the all-reduce path): rank 0 folds the residual, the others
        start from zero, then all-reduce; False: just accumulate this rank's partial into h.
        Expert parallel (replicated tokens): only the pairs routed to this rank's experts run;
        the other pairs weigh 0 in the combine, and the reduction sums the ranks' shares."""
        c = self.cfg
        T, k = xn.shape[0], c.top_k_experts
        w, ids = self._route(xn, Lw)
        if self.w.ep:
            # other ranks' experts: local id -1 / weight 0 on the device; the expert GEMMs skip
            # those pairs (moe_align places no -1 row, GEMV blocks of a -1 pair exit) and the
            # combine skips zero-weight pairs — no host sync, no index kernels
            lids = torch.empty_like(ids)
            lw = torch.empty_like(w)
            ops.moe_ep_localize(ids, w, self.w.e0, self.w.n_local_experts, lids, lw)
            y = self._expert_ffn(xn, lids, Lw)
            w, ids = lw, lids
        else:
            y = self._expert_ffn(xn, ids, Lw)
        if reduce and self.tp.rank != 0:
            h.zero_()
        ops.moe_combine(y, w, ids, h)
        if reduce:
            self.tp.all_reduce_(h)

    def _moe_ep_a2a(self, xs: torch.Tensor, Lw, hs: torch.Tensor) -> None:
        """hs += MoE(xs) for this rank's token shard, experts sharded over the TP group: every
        (token, slot) pair is sent to the rank owning its expert (all-to-all, C4), computed there
        by the grouped GEMM, and sent back for the deterministic combine.

        The plan stays on the device (``moe_ep_dispatch``: stable slots per destination rank, -1
        padding; ``gather_rows`` builds the send buffer), so the layer loop has no host sync: the
        all-to-all moves a fixed ``cap`` = T*k rows per peer (every pair of the shard may pick one
        rank), the receiver's padding rows carry expert id -1 and are skipped by the expert GEMMs,
        and the combine reads each pair's returned row through its slot. The price is padded
        all-to-all traffic (n x the routed rows) for no host round trip per layer."""
        k = self.cfg.top_k_experts
        El, n = self.w.n_local_experts, self.tp.size
        w, ids = self._route(xs, Lw)
        cap = ids.numel()
        send_pair, send_e, slot, _ = ops.moe_ep_dispatch(ids, El, n, cap)
        send_x = ops.gather_rows(xs, send_pair, k)
        split = [cap] * n
        recv_x = self.tp.all_to_all_rows(send_x, split, split)
        recv_e = self.tp.all_to_all_rows(send_e, split, split)
        y_recv = self._expert_ffn(recv_x, recv_e.view(-1, 1), Lw)
        y_back = self.tp.all_to_all_rows(y_recv, split, split)
        ops.moe_combine(y_back, w, ids, hs, rows=slot)

    # -- decode -------------------------------------------------------------------------------------
    def _decode_step(self, B: int, bucket: Optional[int] = None) -> None:
        """One token for rows 0..B-1. ``bucket`` indexes ``attn_buckets`` (default: the largest)."""
        c = self.cfg
        _, chunk, grid_chunks, fused = self.attn_buckets[-1 if bucket is None else bucket]
        part = self.attn_part
        h, q, attn, act = self.h[:B], self.q[:B], self.attn[:B], self.act[:B]
        ops.embedding(self.tokens_in[:B], self.w.embed, out=h)
        bi = -1 if bucket is None else bucket
        ao_chunk = self.ao_chunks[bi] if B == 1 else 0
        qa = self.qa_plan[bi] if B == 1 else None
        dbg = self._debug_layer_io  # eager debug steps only: each layer's input, then the last output
        layers = self.w.layers
        for li, Lw in enumerate(layers):
            if dbg is not None:
                dbg.append(h.clone())
            routed = False
            if qa:  # qkv projection + attention in one launch (one row), then o_proj
                o_in = self.qa_o and h.is_cuda  # ... o_proj (+ all-reduce) in the same launch
                tp = self.tp
                car = tp.custom_fused if (o_in and tp.size > 1 and self.ecfg.fused_ar) else None
                ops.qkv_attn(h, Lw.w_qkv, Lw.ln1, c.rms_eps, q, self.k_cache[li], self.v_cache[li], self.positions[:1],
                             self.slots[:1], self.cos_t, self.sin_t, self.block_tables[:1], self.seq_lens[:1], attn,
                             part, self.attn_counters, self.qa_ws, self.nh, self.nkv, self.D, self.bs, qa[0], qa[1],
                             self.scale, fault=self.attn_fault, w_o=Lw.w_o if o_in else None, h=h if o_in else None,
                             add_resid=tp.rank == 0, car=car)
                if not o_in:
                    self._row_parallel(attn, Lw.w_o, h)
                elif tp.size > 1 and car is None:
                    tp.all_reduce_(h)
            else:
                ops.qkv_rope(h, Lw.w_qkv, Lw.ln1, c.rms_eps, q, self.k_cache[li], self.v_cache[li],
                             self.positions[:B], self.slots[:B], self.cos_t, self.sin_t, self.nh, self.nkv, self.D,
                             self.bs, mfma=self.mfma_decode)
                if ao_chunk:  # one-row engines: attention + o_proj + residual (+ TP all-reduce) in one launch
                    routed = self.ao_router[bi] and h.is_cuda  # ... (+ the MoE router)
                    self._attn_oproj(q, li, Lw, h, attn, ao_chunk, routed)
                else:
                    ops.attn_decode(q, self.k_cache[li], self.v_cache[li], self.block_tables[:B], self.seq_lens[:B],
                                    attn, part[:B], self.attn_counters[:B], self.nh, self.nkv, self.D, self.bs, chunk,
                                    self.scale, grid_chunks, fused=fused, fault=self.attn_fault)
                    self._row_parallel(attn, Lw.w_o, h)
            if c.is_moe:
                self._moe_decode(h, Lw, B, routed)
            else:
                ops.linear(h, Lw.w_gu, EPI_SILU, out=act, norm_w=Lw.ln2, eps=c.rms_eps, mfma=self.mfma_decode)
                self._row_parallel(act, Lw.w_down, h)
        if dbg is not None:
            dbg.append(h.clone())
        self._lm_head_sample(B)

    _debug_layer_io: Optional[list] = None

    def _attn_oproj(self, q, li, Lw, h, attn, chunk, routed: bool = False) -> None:
        """h += o_proj(attention(q)) for one row in one launch (csrc/kernels/attn_oproj.hip). A TP rank
        computes its row-parallel share (rank 0's carries the residual) and all-reduces it inside the
        kernel when the group has the fused buffer (``fused_ar``), else with the group's all-reduce
        launch after it. ``routed``: the MoE layer's router on the new h in the same launch (into
        moe_w / moe_ids, as _moe_decode's router launch would write them)."""
        tp = self.tp
        car = tp.custom_fused if (tp.size > 1 and self.ecfg.fused_ar) else None
        router = None
        if routed:
            router = (Lw.ln2, Lw.w_router, self.cfg.rms_eps, self.cfg.top_k_experts, self.moe_w[:1], self.moe_ids[:1],
                      self.ao_rws)
        ops.attn_oproj(q, self.k_cache[li], self.v_cache[li], self.block_tables[:1], self.seq_lens[:1], Lw.w_o, h, attn,
                       self.ao_ws, self.nh, self.nkv, self.D, self.bs, chunk, self.ao_nc, self.scale,
                       fault=self.attn_fault, add_resid=tp.rank == 0, car=car, router=router)
        if tp.size > 1 and car is None:
            tp.all_reduce_(h)

    @torch.no_grad()
    def debug_decode_layers(self, prompt: Seq[int]):
        """Per-layer hidden states of ONE eager decode step after prefilling ``prompt`` (TP=1, one
        row): (hs [n_layers + 1, H] bf16 — the input of every layer, then the last layer's output —,
        the position of the decoded token). The hook of the per-layer numerics test, which runs an
        fp32 oracle of each layer on the engine's own input and KV cache."""
        if self.tp.size != 1:
            raise EngineError("debug_decode_layers: TP=1 only")
        seq = self.new_sequence()
        try:
            with self._on_stream():
                self.prefill([seq], [list(prompt)])
                self._reserve(seq, seq.length + 4)
                self._use_topkp = False
                self._bind_rows([seq], [SamplingParams(2, 0.0, 1.0, 0, 0, False)])
                self._sample(1, self._gather_logits(1))  # the prefill's token -> this step's input
                pos = int(self.positions[0].item())
                self._debug_layer_io = []
                try:
                    self._decode_step(1, self._bucket(seq.length + 4))
                    hs = torch.cat(self._debug_layer_io)
                finally:
                    self._debug_layer_io = None
            if self.on_gpu:
                self.stream.synchronize()
            return hs, pos
        finally:
            self.free_sequence(seq)

    def _lm_head_sample(self, B: int) -> None:
        lg = self.logits_local[:B]
        ops.linear(self.h[:B], self.w.lm_head, EPI_F32, out=lg, norm_w=self.w.final_norm, eps=self.cfg.rms_eps,
                   mfma=self.mfma_decode)
        logits = self._gather_logits(B)
        self._sample(B, logits)

    def _moe_decode(self, h, Lw, B, routed: bool = False) -> None:
        """``routed``: the fused attention + o_proj launch already wrote moe_w / moe_ids."""
        c = self.cfg
        if not h.is_cuda:
            xn = self.xn[:B]
            ops.rmsnorm(h, Lw.ln2, c.rms_eps, out=xn)
            self._moe(xn, Lw, h)
            return
        k = c.top_k_experts
        w, ids = self.moe_w[:B], self.moe_ids[:B]
        # one launch: rmsnorm -> router logits -> top-k; the expert gate_up GEMV normalises h
        # again in its own prologue, so the normed row never goes through memory
        if not routed:
            ops.moe_router(h, Lw.ln2, c.rms_eps, Lw.w_router, k, w, ids)
        if self.w.ep:  # pairs of other ranks' experts: id -1 (GEMV blocks exit), weight 0
            ops.moe_ep_localize(ids, w, self.w.e0, self.w.n_local_experts, self.moe_lids[:B], self.moe_lw[:B])
            w, ids = self.moe_lw[:B], self.moe_lids[:B]
        I_l, H = self.w.inter, c.hidden
        act, y = self.moe_act[: B * k], self.moe_y[: B * k]
        if self.mfma_decode and H % 128 == 0 and I_l % 128 == 0:
            # a batching engine (see mfma_decode): the pairs grouped by expert on the MFMA form, each
            # routed expert streamed once for all its rows, then the combine
            ops.moe_gemvm(h, Lw.w_gu, ids, k, act, 2 * I_l, H, EPI_SILU, norm_w=Lw.ln2, eps=c.rms_eps)
            ops.moe_gemvm(act, Lw.w_down, ids, 1, y, H, I_l, EPI_BF16)
            if self.tp.rank != 0:
                h.zero_()
            ops.moe_combine(y, w, ids, h)
            self.tp.all_reduce_(h)
            return
        ops.moe_gemv(h, Lw.w_gu, ids, k, act, 2 * I_l, H, EPI_SILU, norm_w=Lw.ln2, eps=c.rms_eps)
        if self.tp.rank != 0:  # row-parallel partial: only rank 0 carries the residual
            h.zero_()
        if k == 2 and not self.w.ep:
            # down projection + combine in one launch (each wave streams its row of both experts)
            ops.moe_down_combine(act, Lw.w_down, ids, w, h, H, I_l)
        else:
            ops.moe_gemv(act, Lw.w_down, ids, 1, y, H, I_l, EPI_BF16)
            ops.moe_combine(y, w, ids, h)
        self.tp.all_reduce_(h)

    def _gather_logits(self, B: int) -> torch.Tensor:
        """Vocab-parallel lm_head: all-gather [B, V/tp] shards into [B, V] (C3)."""
        if self.tp.size == 1:
            return self.logits_local[:B]
        n = self.tp.size * B * self.w.vocab_local
        buf = self._gather_buf.view(-1)[:n].view(self.tp.size, B, self.w.vocab_local)
        self.tp.all_gather_rows(self.logits_local[:B], buf)
        out = self.logits[:B]
        if B == 1:
            out.view(-1).copy_(buf.view(-1))
        else:
            out.view(B, self.tp.size, self.w.vocab_local).copy_(buf.permute(1, 0, 2))
        return out

    def full_logits(self, seq: Sequence) -> torch.Tensor:
        """Full-vocabulary last-token logits of a prefilled sequence (collective under TP), safe to
        use on the caller's stream: the prefill ran on the engine's stream and returned without a
        sync, so the gather runs there too and the caller's stream then waits for it (reading
        ``seq.logits`` from another stream raced the prefill's lm_head: a TP=2 test saw a few
        logits not yet written)."""
        if self.tp.size == 1:
            out = seq.logits
        else:
            with self._on_stream():
                self.logits_local[0].copy_(seq.logits)
                out = self._gather_logits(1)[0]
        if self.stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
        return out

    def _sample(self, B: int, logits: torch.Tensor) -> None:
        use_topkp = bool(self._use_topkp)
        ops.sample(logits, self.inv_temp[:B], self.top_k[:B], self.top_p[:B], self.seeds[:B], self.positions[:B],
                   self.next_tok[:B], self.ws_v[:B] if self.ws_v is not None else None,
                   self.ws_i[:B] if self.ws_i is not None else None, tokens_in=self.tokens_in[:B],
                   seq_lens=self.seq_lens[:B], slots=self.slots[:B], block_tables=self.block_tables[:B], bs=self.bs,
                   out_tokens=self.out_tokens[:B], out_count=self.out_count[:B], use_topkp=use_topkp)

    def _bucket(self, ctx_tokens: int) -> int:
        """Smallest attention bucket covering ``ctx_tokens`` (so a short context's graph does not
        launch thousands of empty blocks)."""
        for i, (cap, _, _, _) in enumerate(self.attn_buckets):
            if cap >= ctx_tokens:
                return i
        return len(self.attn_buckets) - 1

    def buckets(self) -> List[int]:
        return list(range(len(self.attn_buckets)))

    @torch.no_grad()
    def warmup_graphs(self, batch_sizes: Optional[List[int]] = None, topkp: bool = False) -> int:
        """Capture every decode graph this engine can need (per batch size x context bucket) up
        front. A process hosting several engines must do this before serving: a capture running
        beside another engine's work is invalidated by HIP, so serving never captures
        (``capture_on_demand`` False -> a missing graph runs eagerly)."""
        if not (self.on_gpu and self.ecfg.use_graphs):
            return 0
        n = 0
        # TP: every rank starts its warm-up steps (eager, with collectives) together — a rank still
        # warming another engine would otherwise hold its peers' spins past their 1-s bound — and
        # leaves it with the collectives' protocol state re-synchronised
        self.tp.barrier()
        with self._on_stream():
            for B in batch_sizes or list(range(1, self.ecfg.max_batch + 1)):
                for bk in self.buckets():
                    self._use_topkp = topkp
                    self._graph(B, bk)
                    n += 1
        self._use_topkp = False
        self.capture_on_demand = False
        if self.tp.size > 1:
            self.stream.synchronize()
            self.tp.resync_collectives()
        return n

    capture_on_demand = True

    def _graph(self, B: int, bucket: int):
        key = (B, self._use_topkp, bucket)
        g = self._graphs.get(key)
        if g is not None or not self.capture_on_demand:
            return g
        S = self.ecfg.steps_per_graph
        # warm up once eagerly (kernel attributes, lazy module state) with the device state
        # snapshotted and restored, then capture S steps.
        snap = self._snapshot_state()
        self._decode_step(B, bucket)
        self._restore_state(snap)
        self.stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=self.stream, capture_error_mode="thread_local"):
            for _ in range(S):
                self._decode_step(B, bucket)
        self._graphs[key] = g
        return g

    _use_topkp = False

    def _snapshot_state(self):
        return [t.clone() for t in (self.tokens_in, self.positions, self.seq_lens, self.slots, self.out_tokens,
                                    self.out_count, self.next_tok)]

    def _restore_state(self, snap) -> None:
        for dst, src in zip((self.tokens_in, self.positions, self.seq_lens, self.slots, self.out_tokens,
                             self.out_count, self.next_tok), snap):
            dst.copy_(src)

    @torch.no_grad()
    def decode(self, seqs: List[Sequence], params: List[SamplingParams], ctx: Optional[Context] = None,
               on_tokens: Optional[Callable[[int, List[int]], None]] = None) -> List[List[int]]:
        """Sample from each sequence's prefill logits, then decode until every row hits max_tokens /
        EOS. ``on_tokens(i, new_ids)`` streams tokens (i indexes ``seqs``). Rows must be 0..B-1."""
        B = len(seqs)
        if B > self.ecfg.max_batch:
            raise EngineError(f"{B} sequences > max_batch {self.ecfg.max_batch}")
        self._check_usable()
        S = self.ecfg.steps_per_graph
        eos_set = set(self.cfg.eos)
        with self._on_stream(), trace.span("decode", engine=self.name, rows=B):
            max_new = max(p.max_tokens for p in params)
            self._use_topkp = any((p.top_k > 0 or p.top_p < 1.0) for p in params)
            for i, (s, p) in enumerate(zip(seqs, params)):
                if not s.has_logits:
                    raise EngineError("sequence has no prefill logits")
                self._reserve(s, s.length + p.max_tokens + S + 1)
            self._bind_rows(seqs, params)
            if max_new > self.cap - S - 1:
                raise EngineError("max_tokens exceeds engine capacity")
            # first token from the prefill logits (+ device state advance)
            self._sample(B, self._gather_logits(B))
            produced = [0] * B
            done = [False] * B
            results: List[List[int]] = [[] for _ in range(B)]
            issued = 1

            def consume(counts, toks) -> None:
                for i in range(B):
                    r = seqs[i].row
                    if done[i]:
                        continue
                    n = min(int(counts[r]), params[i].max_tokens)
                    new = toks[r][produced[i]:n].tolist() if n > produced[i] else []
                    stop = False
                    hit = next((j for j, t in enumerate(new) if t in eos_set), -1) if params[i].stop_on_eos else -1
                    if hit >= 0:
                        new = new[:hit]
                        stop = True
                    if new:
                        results[i].extend(new)
                        if on_tokens:
                            on_tokens(i, new)
                    produced[i] = n if not stop else produced[i] + len(new)
                    if stop or n >= params[i].max_tokens:
                        done[i] = True

            tp_ctl = self.tp.size > 1 and self.tp.ctrl is not None
            failure: Optional[BaseException] = None

            def agree() -> bool:
                """After each consumed snapshot: True = every row is finished. Raises on a
                cancellation (the leader's) or a failure anywhere in the TP group — on every rank at
                the same replay (TPGroup.step_agree), after draining and checking the collectives."""
                if tp_ctl:
                    try:
                        stop, failed, fin = self.tp.step_agree(self._ctx_done(ctx), failure is not None, all(done))
                    except Exception as e:  # noqa: BLE001 - the control group itself failed (peer died)
                        self._tp_broken(f"{type(e).__name__}: {e}")
                    if failed:
                        self._fail_tp(failure)
                else:
                    fin, stop = all(done), False
                    if not fin:
                        stop = self._stop_requested(ctx)
                if fin:
                    return True
                if stop:
                    self._drain()
                    self._check_collectives()
                    raise ContextError(self._stop_reason(ctx))
                return False

            if not self.on_gpu:
                while True:
                    try:
                        self._inject("decode", issued)
                        consume(self.out_count, self.out_tokens)
                    except Exception as e:  # noqa: BLE001
                        if not tp_ctl:
                            raise
                        failure = e
                    if agree():
                        break
                    self._decode_step(B)
                    issued += 1
                self._check_collectives()
                self._finish(seqs, results)
                return results

            base_len = max(s.length for s in seqs)
            pending_ev: Optional[torch.cuda.Event] = None

            def launch_copy(upto: int):
                # only the token window produced since the last snapshot travels (columns
                # [lo, upto) of every row; earlier columns are already in the host copy)
                lo = min(produced) if produced else 0
                hi = min(self.cap, upto)
                self.host_count[:B].copy_(self.out_count[:B], non_blocking=True)
                if hi > lo:  # per row: contiguous spans, so the copies stay asynchronous
                    for r in range(B):
                        self.host_tokens[r, lo:hi].copy_(self.out_tokens[r, lo:hi], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
                return ev

            if self.tp.size > 1:
                # the prefill and the first sample finish before the replay deadline clock starts
                # (a long TP prefill is not a stalled replay: ADVICE r5); its collectives' spins are
                # bounded, so this wait is too
                self.stream.synchronize()
            self._replay_aborted = False
            pending_ev = launch_copy(issued)
            last = False
            while True:
                need_more = issued < max_new
                try:
                    if need_more and failure is None:
                        self._inject("decode", issued)
                        # context reached by the end of this replay decides the attention bucket
                        bucket = self._bucket(base_len + issued + S + 1)
                        graph = self._graph(B, bucket) if self.ecfg.use_graphs else None
                        if graph is not None:
                            graph.replay()
                        else:
                            for _ in range(S):
                                self._decode_step(B, bucket)
                        issued += S
                    # wait for the previous snapshot (the GPU keeps the just-issued replay queued)
                    self._wait_event(pending_ev)
                    # a custom-collective spin that gave up (or a host abort) invalidates every later
                    # collective result: fail before these tokens are streamed, not at the end
                    self._raise_if_collectives_gave_up()
                    consume(self.host_count, self.host_tokens)
                except Exception as e:  # noqa: BLE001 - under TP: agreed below, on every rank
                    if not tp_ctl or isinstance(e, _TPBroken):
                        raise
                    failure = e
                # every TP rank takes this decision identically, at the same replay: one rank
                # running an extra replay would desynchronise the collectives
                if agree() or last:
                    break
                pending_ev = launch_copy(issued)
                last = not need_more
            self._drain()
            self._check_collectives()
            self._finish(seqs, results)
            return results

    # -- TP failure handling ------------------------------------------------------------------------
    # Seconds a TP engine waits for a replay's snapshot before it aborts its custom-collective spins
    # (a peer stalled or died: the device spins give up on their own after 1 s, so this only fires
    # when they cannot, e.g. an RCCL fallback collective), and again before it declares the device
    # stalled. LLMC_TP_STALL_S.
    stall_s = float(os.environ.get("LLMC_TP_STALL_S", "5"))

    def _wait_event(self, ev) -> None:
        """Wait for ``ev``: a plain synchronize without TP peers; a TP engine polls it against a
        deadline instead, so a replay stuck on a peer cannot block the host indefinitely."""
        if self.tp.size == 1 or not self.on_gpu:
            ev.synchronize()
            return
        deadline, aborted = time.monotonic() + self.stall_s, False
        while not ev.query():
            if time.monotonic() > deadline:
                if aborted:
                    self._tp_broken(f"a decode replay did not finish {2 * self.stall_s:.0f} s after it was due "
                                    "(its collectives were aborted)")
                self.tp.abort_collectives()  # the spins give up at their next check
                self._replay_aborted = True
                deadline, aborted = time.monotonic() + self.stall_s, True
            time.sleep(0.0002)

    _replay_aborted = False

    def _raise_if_collectives_gave_up(self) -> None:
        """Under TP: raise if a custom-collective spin of this rank gave up or returned without its
        data since the last resync (the host status page: no GPU call, the stream keeps running), or
        the host aborted a replay — from then on every collective of this rank returns at once with
        stale data, so no later token may be streamed. The decode loop turns it into the
        agreed failure of the group at this replay."""
        if self.tp.size == 1:
            return
        if self._replay_aborted or any(c.host_timed_out() for c in self.tp.collectives()):
            raise EngineError("custom all-reduce gave up on a stalled TP peer: this request's later tokens "
                              "would be invalid")

    def _drain(self) -> None:
        """The stream's queued work finished (bounded under TP, see ``_wait_event``)."""
        if self.on_gpu:
            ev = torch.cuda.Event()
            ev.record(self.stream)
            self._wait_event(ev)

    def _fail_tp(self, failure: Optional[BaseException]) -> None:
        """A rank of the TP group failed mid-decode (agreed by every rank at the same replay): the
        replays every rank launched pair up, so drain them, check / re-synchronise the collectives
        (a rank whose replays stopped made its peers' spins give up), then raise — the failed rank
        its own error, the others an EngineError (reference runner.go:100-107: that model fails,
        the run goes on)."""
        self._drain()
        try:
            self._check_collectives()
        except EngineError:
            pass
        if failure is not None:
            raise failure
        raise EngineError("a TP peer failed mid-decode: this request is failed on every rank of the group")

    def _tp_broken(self, why: str) -> None:
        """The group can no longer agree (a peer process died, a control round or a device wait
        timed out): abort this rank's spins, mark the group broken (every later request fails at
        once) and fail the request."""
        self.tp.broken = why
        self.tp.abort_collectives()
        raise _TPBroken(f"TP group broken: {why}")

    def _inject(self, stage: str, issued: int) -> None:
        """Test hook (SURVEY.md §5.3 fault injection): ``fault_at`` = (stage, k) raises an
        InjectedEngineFault before the decode replay that would produce token k (its peers' replays
        then wait on this rank's collectives until their spins give up); (stage, k, seconds) stalls
        the rank that long there instead, then lets it go on."""
        f = self.fault_at
        if f is not None and f[0] == stage and issued >= f[1]:
            self.fault_at = None
            if len(f) > 2:  # (stage, k, seconds): a rank that stalls, then goes on
                time.sleep(float(f[2]))
                return
            raise InjectedEngineFault(f"injected fault: {self.name} stops before decode token {issued}")

    fault_at: Optional[tuple] = None

    def _check_usable(self) -> None:
        if self.tp.broken:
            raise EngineError(f"{self.name}: TP group broken ({self.tp.broken}); the engine serves no more requests")

    # -- TP control plane -------------------------------------------------------------------------
    @staticmethod
    def _ctx_done(ctx: Optional[Context]) -> bool:
        return ctx is not None and ctx.done()

    def _stop_requested(self, ctx: Optional[Context]) -> bool:
        """Cancellation / deadline between replays. Under TP with a control group the TP leader's
        context decides for every rank (a follower's own cancel arrives at its own time)."""
        local = ctx is not None and ctx.done()
        if self.tp.size > 1 and self.tp.ctrl is not None:
            return bool(self.tp.leader_decides(int(local), "stop"))
        return local

    @staticmethod
    def _stop_reason(ctx: Optional[Context]) -> str:
        return (ctx.err() if ctx is not None else None) or "context canceled"

    def _check_collectives(self) -> None:
        """After a decode (stream synchronised): fail the request if a bounded device spin gave up
        since the last check, on every rank of a TP group with a control group.

        * custom-collective spins: the group re-synchronises its protocol state first, so the next
          request runs on consistent epochs;
        * decode-attention merges (``attn_fault``): a merger that gave up merged a partial that
          never arrived, so the tokens sampled from it are wrong — reported, never streamed on
          silently (reference ``runner.go:100-107`` reports failures)."""
        attn_bad = False
        if self.attn_fault is not None:
            attn_bad = bool(self.attn_fault.item())
            if attn_bad:
                self.attn_fault.zero_()
        if self.tp.size > 1 and self.tp.ctrl is not None:
            if not self.tp.check_collectives():
                raise EngineError("custom all-reduce timed out (a TP peer stalled): this request's tokens are invalid")
            attn_bad = self.tp.any_rank(attn_bad)
        if attn_bad:
            raise EngineError("decode attention: a partial merge timed out (a block never published its "
                              "partial, or an attention + o_proj hand-off wait gave up): this "
                              "request's tokens are invalid")

    def _bind_rows(self, seqs: List[Sequence], params: List[SamplingParams]) -> None:
        """Bind sequences to decode rows 0..B-1: block tables, prefill logits and sampling state."""
        B = len(seqs)
        self.block_tables[:B].copy_(self._block_table(seqs))
        for i, (s, p) in enumerate(zip(seqs, params)):
            s.row = i
            self.logits_local[i].copy_(s.logits)
            self.inv_temp[i] = 0.0 if p.temperature <= 0 else 1.0 / p.temperature
            self.top_k[i] = p.top_k
            self.top_p[i] = p.top_p
            self.seeds[i] = p.seed
            self.positions[i] = s.length - 1
            self.out_count[i] = 0

    @torch.no_grad()
    def debug_decode_logits(self, prompt: Seq[int], n: int):
        """Greedy decode of ``n`` tokens one eager step at a time (TP=1), returning (tokens, logits
        [n, V] f32): row i holds the full-vocabulary logits token i was sampled from — the hook the
        teacher-forced oracle test compares against a CPU prefill of prompt + tokens[:i]."""
        toks, lg = self.debug_decode_logits_batch([prompt], n)
        return toks[0], lg[0]

    @torch.no_grad()
    def debug_decode_logits_batch(self, prompts: List[Seq[int]], n: int):
        """``debug_decode_logits`` for B = len(prompts) rows decoded together (the batched decode
        GEMV forms: VALU rows <= 2, MFMA 3-32): (tokens [B][n], logits [B, n, V] f32)."""
        if self.tp.size != 1:
            raise EngineError("debug_decode_logits: TP=1 only")
        B = len(prompts)
        if B > self.ecfg.max_batch:
            raise EngineError(f"{B} rows > max_batch {self.ecfg.max_batch}")
        seqs = [self.new_sequence() for _ in range(B)]
        try:
            with self._on_stream():
                self.prefill(seqs, [list(p) for p in prompts])
                for s in seqs:
                    self._reserve(s, s.length + n + 2)
                self._use_topkp = False
                self._bind_rows(seqs, [SamplingParams(n, 0.0, 1.0, 0, 0, False)] * B)
                rows = [self.logits_local[:B].clone()]
                self._sample(B, self._gather_logits(B))
                bucket = self._bucket(max(s.length for s in seqs) + n + 2)
                for _ in range(n - 1):
                    self._decode_step(B, bucket)
                    rows.append(self.logits_local[:B].clone())
                toks = self.out_tokens[:B, :n].clone()
            if self.on_gpu:
                self.stream.synchronize()
            return toks.cpu().tolist(), torch.stack(rows, 1).float().cpu()
        finally:
            for s in seqs:
                self.free_sequence(s)

    def _finish(self, seqs, results) -> None:
        for s, r in zip(seqs, results):
            s.length += len(r)
            s.has_logits = False

    def _eos_id(self) -> int:
        return self.cfg.eos[0]

    # -- convenience ----------------------------------------------------------------------------------
    @torch.no_grad()
    def generate_ids(self, prompt: Seq[int], max_tokens: int, temperature: float = 1.0, top_p: float = 1.0,
                     top_k: int = 0, seed: int = 0, stop_on_eos: bool = True, ctx: Optional[Context] = None,
                     on_tokens: Optional[Callable[[List[int]], None]] = None) -> List[int]:
        seq = self.new_sequence()
        try:
            self.prefill([seq], [list(prompt)])
            p = SamplingParams(max_tokens, temperature, top_p, top_k, seed, stop_on_eos)
            cb = (lambda i, ids: on_tokens(ids)) if on_tokens else None
            return self.decode([seq], [p], ctx, cb)[0]
        finally:
            self.free_sequence(seq)

    @torch.no_grad()
    def generate_batch(self, prompts: List[List[int]], params: List[SamplingParams], ctx: Optional[Context] = None,
                       on_tokens=None) -> List[List[int]]:
        seqs = [self.new_sequence() for _ in prompts]
        try:
            self.prefill(seqs, prompts)
            return self.decode(seqs, params, ctx, on_tokens)
        finally:
            for s in seqs:
                self.free_sequence(s)

    def synchronize(self) -> None:
        if self.stream is not None:
            self.stream.synchronize()

    def memory_bytes(self) -> int:
        return self.w.nbytes() + 2 * self.k_cache.numel() * 2
