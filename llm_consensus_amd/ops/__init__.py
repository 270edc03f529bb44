"""Op layer: one entry point per kernel.

CUDA (ROCm) tensors → hand-written gfx950 HIP kernels in ``_llmc_hip`` (raises if the module is
missing: there is no silent PyTorch fallback on the GPU). CPU tensors → ``oracle`` (reference
semantics; used by CPU tests of model/TP/engine logic). All launches go to torch's current
stream, so every op is capturable in a HIP graph.
"""

from __future__ import annotations

import os
from typing import Optional

import torch

from ..utils.native import kernels
from . import oracle

EPI_BF16, EPI_F32, EPI_RESADD, EPI_SILU, EPI_ROPE = 0, 1, 2, 3, 4
GEMV_MAX_M = 32      # decode rows on the weight-streaming path (VALU GEMV 1-2, MFMA form 3-32)
MOE_GEMVM_MAX_TOKENS = 16  # batched MoE decode: (token, expert) pairs of <= 16 tokens per launch
MOE_GEMV_MAX_M = 4   # MoE: per-(row, expert) GEMVs up to this many rows, then the grouped GEMM


def _p(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def _s(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _bf16(t: torch.Tensor, name: str) -> None:
    if t.dtype != torch.bfloat16:
        raise TypeError(f"{name}: expected bfloat16, got {t.dtype}")


# ---------------------------------------------------------------------------------------------
def lane_exchange_check(x: torch.Tensor) -> torch.Tensor:
    """GPU self-test of the kernels' cross-lane helpers (csrc/kernels/common.h: v_permlane*_swap and
    DPP forms of the wave reductions). ``x``: f32 [nb * 64] on the GPU; returns f32 [nb * 64, 10, 2]:
    (helper, __shfl_xor form) pairs that must match bit for bit."""
    if not x.is_cuda:
        raise RuntimeError("lane_exchange_check: GPU only")
    x = x.contiguous().float()
    nb = x.numel() // 64
    out = torch.empty(nb * 64, 10, 2, dtype=torch.float32, device=x.device)
    kernels().lane_exchange_check(_p(x), _p(out), nb, _s(x))
    return out


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not x.is_cuda:
        r = oracle.rmsnorm(x, w, eps)
        return out.copy_(r) if out is not None else r
    _bf16(x, "rmsnorm.x")
    H = x.shape[-1]
    x2 = x.reshape(-1, H)
    if out is None:
        out = torch.empty_like(x)
    kernels().rmsnorm(_p(x2), _p(w), _p(out), x2.shape[0], H, x2.stride(0), out.reshape(-1, H).stride(0), float(eps), _s(x))
    return out


def embedding(ids: torch.Tensor, table: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not table.is_cuda:
        r = oracle.embedding(ids, table)
        return out.copy_(r) if out is not None else r
    T = ids.numel()
    if out is None:
        out = torch.empty(T, table.shape[1], dtype=table.dtype, device=table.device)
    kernels().embedding(_p(ids), _p(table), _p(out), T, table.shape[1], table.shape[0], _s(table))
    return out


def silu_mul_interleaved(gu: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not gu.is_cuda:
        r = oracle.silu_mul_interleaved(gu)
        return out.copy_(r) if out is not None else r
    T, I2 = gu.shape
    if out is None:
        out = torch.empty(T, I2 // 2, dtype=gu.dtype, device=gu.device)
    kernels().silu_mul_interleaved(_p(gu), _p(out), T, I2 // 2, _s(gu))
    return out


def linear(x: torch.Tensor, W: torch.Tensor, epi: int = EPI_BF16, out: Optional[torch.Tensor] = None,
           norm_w: Optional[torch.Tensor] = None, eps: float = 1e-5, mfma: bool = False) -> torch.Tensor:
    """y = (rmsnorm(x)*norm_w if norm_w else x) @ W^T with a fused epilogue.

    M <= 32 rows -> weight streaming (decode; the norm runs in its prologue): the VALU GEMV for 1-2
    rows, the MFMA form for 3-32 (one 16-token column group up to 16 rows, two above) (``mfma`` pins the MFMA form at every row count: a batching
    engine's decode stays batch-invariant); larger M -> the 256x256 MFMA prefill GEMM
    (csrc/kernels/gemm.hip; a norm is a separate rmsnorm launch first).
    Epilogues: bf16 | f32 | EPI_RESADD (accumulates into ``out`` in place) | EPI_SILU (interleaved
    gate/up columns -> silu(g) * u, [M, N / 2]). One code path per shape class, all hand-written.
    """
    if not x.is_cuda:
        return oracle.linear(x, W, epi, out, norm_w, eps)
    _bf16(x, "linear.x")
    _bf16(W, "linear.W")
    M, K = x.shape
    N = W.shape[0]
    if W.shape[1] != K:
        raise ValueError(f"linear: x[{M},{K}] vs W{tuple(W.shape)}")
    if out is None:
        if epi == EPI_RESADD:
            raise ValueError("EPI_RESADD needs out")
        n_out = N // 2 if epi == EPI_SILU else N
        out = torch.empty(M, n_out, dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16, device=x.device)
    if M <= 4 or (M <= GEMV_MAX_M and K % 128 == 0 and x.stride(0) % 8 == 0):
        kernels().gemv(M, _p(x), x.stride(0), _p(norm_w), float(eps), _p(W), _p(out), out.stride(0), N, K, epi,
                       int(mfma), _s(x))
        return out
    if norm_w is not None:
        x = rmsnorm(x, norm_w, eps)
    kernels().gemm(_p(x), x.stride(0), _p(W), W.stride(0), _p(out), out.stride(0), M, N, K, epi, _s(x))
    return out


def gemm(x: torch.Tensor, W: torch.Tensor, epi: int = EPI_BF16, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Always the MFMA GEMM path, kernel chosen by ``gemm_plan`` (tests / microbenchmarks)."""
    if not x.is_cuda:
        return oracle.linear(x, W, epi, out)
    M, K = x.shape
    N = W.shape[0]
    if out is None:
        n_out = N // 2 if epi == EPI_SILU else N
        out = torch.empty(M, n_out, dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16, device=x.device)
    kernels().gemm(_p(x), x.stride(0), _p(W), W.stride(0), _p(out), out.stride(0), M, N, K, epi, _s(x))
    return out


def gemm128(x: torch.Tensor, W: torch.Tensor, epi: int = EPI_BF16, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Always the 128 x 128 two-buffer MFMA kernel (tests / microbenchmarks of the narrow-N choice)."""
    if not x.is_cuda:
        return oracle.linear(x, W, epi, out)
    M, K = x.shape
    N = W.shape[0]
    if out is None:
        n_out = N // 2 if epi == EPI_SILU else N
        out = torch.empty(M, n_out, dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16, device=x.device)
    kernels().gemm_t128(_p(x), x.stride(0), _p(W), W.stride(0), _p(out), out.stride(0), M, N, K, epi, _s(x))
    return out


def _gemm_kind(x, W, epi, out, kind):
    if not x.is_cuda:
        return oracle.linear(x, W, epi, out)
    M, K = x.shape
    N = W.shape[0]
    if out is None:
        n_out = N // 2 if epi == EPI_SILU else N
        out = torch.empty(M, n_out, dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16, device=x.device)
    kernels().gemm_kind(_p(x), x.stride(0), _p(W), W.stride(0), _p(out), out.stride(0), M, N, K, epi, kind, _s(x))
    return out


def gemm256(x: torch.Tensor, W: torch.Tensor, epi: int = EPI_BF16, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Always the 256 x 256 LDS-DMA ring kernel (tests / microbenchmarks)."""
    return _gemm_kind(x, W, epi, out, 0)


def gemm_narrow(x: torch.Tensor, W: torch.Tensor, epi: int = EPI_BF16, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Always the 128 x 192 narrow-N MFMA kernel (tests / microbenchmarks of the narrow-N dispatch)."""
    return _gemm_kind(x, W, epi, out, 1)


def gemm_plan(M: int, N: int) -> str:
    """The prefill GEMM kernel ``linear`` / ``gemm`` launch for a dense [M, N] output (host-side model,
    csrc/kernels/gemm.hip ``llmc_gemm_plan``): "256x256" or "128x192"."""
    return ("256x256", "128x192")[kernels().gemm_plan(int(M), int(N))]


def gemv(x: torch.Tensor, W: torch.Tensor, epi: int = EPI_BF16, out: Optional[torch.Tensor] = None,
         norm_w: Optional[torch.Tensor] = None, eps: float = 1e-5, mfma: bool = False) -> torch.Tensor:
    """Always the weight-streaming path (M <= 32; the kernel library picks VALU / MFMA form)."""
    if not x.is_cuda:
        return oracle.linear(x, W, epi, out, norm_w, eps)
    M, K = x.shape
    N = W.shape[0]
    if out is None:
        n_out = N // 2 if epi == EPI_SILU else N
        out = torch.empty(M, n_out, dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16, device=x.device)
    kernels().gemv(M, _p(x), x.stride(0), _p(norm_w), float(eps), _p(W), _p(out), out.stride(0), N, K, epi, int(mfma),
                   _s(x))
    return out


def gemvm(x: torch.Tensor, W: torch.Tensor, epi: int = EPI_BF16, out: Optional[torch.Tensor] = None,
          norm_w: Optional[torch.Tensor] = None, eps: float = 1e-5, form: int = 0) -> torch.Tensor:
    """Always the MFMA weight-streaming form (gemv_mfma.hip; M <= 32) — tests / microbenchmarks
    (``linear``/``gemv`` take it by themselves for 3 <= M <= 32). ``form`` 0 = by shape, 1-4 pin
    (row groups per wave, x path) = (1, L2), (1, LDS), (2, L2), (2, LDS)."""
    if not x.is_cuda:
        return oracle.linear(x, W, epi, out, norm_w, eps)
    M, K = x.shape
    N = W.shape[0]
    if out is None:
        n_out = N // 2 if epi == EPI_SILU else N
        out = torch.empty(M, n_out, dtype=torch.float32 if epi == EPI_F32 else torch.bfloat16, device=x.device)
    kernels().gemvm(M, _p(x), x.stride(0), _p(norm_w), float(eps), _p(W), _p(out), out.stride(0), N, K, epi, form,
                    _s(x))
    return out


def rope_kv_write(qkv, positions, cos_t, sin_t, k_cache, v_cache, slots, nh, nkv, D, bs, q_out) -> None:
    """Prefill RoPE: pair-interleaved Q/K rows of ``qkv`` -> canonical rotated q in ``q_out``,
    rotated k and raw v into the paged cache."""
    if not qkv.is_cuda:
        oracle.rope_kv_write(qkv, positions, cos_t, sin_t, k_cache, v_cache, slots, nh, nkv, D, bs, q_out)
        return
    T = qkv.shape[0]
    kernels().rope_kv_write(_p(qkv), qkv.stride(0), _p(q_out), q_out.stride(0), _p(positions), _p(cos_t), _p(sin_t),
                            _p(k_cache), _p(v_cache), _p(slots), T, nh, nkv, D, bs, _s(qkv))


def qkv_rope(x, W, norm_w, eps, q_out, k_cache, v_cache, positions, slots, cos_t, sin_t, nh, nkv, D, bs,
             mfma: bool = False) -> None:
    """Decode qkv projection: fused RMSNorm prologue + RoPE/KV-write epilogue (one launch; form as
    ``linear``)."""
    if not x.is_cuda:
        qkv = oracle.linear(x, W, EPI_BF16, None, norm_w, eps)
        oracle.rope_kv_write(qkv, positions, cos_t, sin_t, k_cache, v_cache, slots, nh, nkv, D, bs, q_out)
        return
    M, K = x.shape
    if M > 4 and (K % 128 != 0 or x.stride(0) % 8 != 0):  # outside the MFMA decode form: prefill's path
        qkv = linear(x, W, EPI_BF16, norm_w=norm_w, eps=eps)
        rope_kv_write(qkv, positions, cos_t, sin_t, k_cache, v_cache, slots, nh, nkv, D, bs, q_out)
        return
    kernels().gemv_qkv_rope(M, _p(x), x.stride(0), _p(norm_w), float(eps), _p(W), W.shape[0], K, _p(q_out),
                            q_out.stride(0), _p(k_cache), _p(v_cache), _p(positions), _p(slots), _p(cos_t), _p(sin_t),
                            nh, nkv, D, bs, int(mfma), _s(x))


FUSED_ATTN_MAX_KEYS = 4096  # decode attention: fused single-launch form up to this bucket capacity
FUSED_CHUNK = 128           # keys per block of the fused form


ATTN_CTR_PITCH = 32  # int32 words per decode-attention counter line (attn_core.h kCtrPitch)


def decode_attn_workspace(B, nh, nkv, D, max_chunks, device, fused: bool = False):
    """(part, counters) for attn_decode, either form: partial granules f32 [B, nkv, max_chunks +
    groups, G, D + 4] (bf16 {value pair, tag} granules merged in-launch; the extra rows hold the
    group results of a two-level merge) and the per-(row, kv head) {top ticket, epoch, group
    tickets} int32 [B, nkv, 2 + groups, ATTN_CTR_PITCH] (one 128-B line per word: returning atomics
    on one line serialise), both zeroed once and never reset (the kernel re-arms the
    tickets and advances the epochs). ``groups`` comes from the kernel library
    (``llmc_attn_decode_groups``). ``fused`` is accepted for call-site symmetry."""
    G = nh // nkv
    dev = torch.device(device)
    groups = kernels().attn_decode_groups(max_chunks) if dev.type == "cuda" else 0  # CPU: oracle path
    part = torch.zeros(B, nkv, max_chunks + groups, G, D + 4, dtype=torch.float32, device=dev)
    counters = torch.zeros(B, nkv, 2 + groups, ATTN_CTR_PITCH, dtype=torch.int32, device=dev)
    return part, counters


def attn_decode(q, k_cache, v_cache, block_tables, seq_lens, out, part, counters, nh, nkv, D, bs, chunk, scale,
                grid_chunks: Optional[int] = None, fused: bool = False, fault: Optional[torch.Tensor] = None):
    """Decode attention (K5), one launch. ``fused``: fixed ``chunk``-key blocks (128 or 256;
    ``grid_chunks`` = bucket capacity / chunk) — short contexts; else the balanced split over <=
    grid_chunks 8-wave blocks of >= ``chunk`` keys — long contexts. Both merge their partials in
    the same launch. ``part``/``counters`` come from ``decode_attn_workspace``. ``fault`` (int32
    [1], optional) is set to 1 by a merger that gave up waiting for a partial (bounded spin): the
    output is then invalid (``Engine`` checks it after every decode and fails the request)."""
    if not q.is_cuda:
        out.copy_(oracle.attn_decode(q, k_cache, v_cache, block_tables, seq_lens, nh, nkv, D, bs, scale))
        return out
    B = q.shape[0]
    groups = counters.shape[-2] - 2
    max_chunks = part.shape[2] - groups
    gc = max_chunks if grid_chunks is None else min(grid_chunks, max_chunks)
    if (part.shape[-1] != D + 4 or counters.shape[0] < B or groups < 0 or counters.shape[-1] != ATTN_CTR_PITCH
            or kernels().attn_decode_groups(max_chunks) != groups):
        raise ValueError("attn_decode: workspace does not match (use decode_attn_workspace)")
    kernels().attn_decode(_p(q), q.stride(0), _p(k_cache), _p(v_cache), _p(block_tables), block_tables.stride(0),
                          _p(seq_lens), _p(part), _p(counters), _p(out), out.stride(0), B, nh, nkv, D, bs,
                          k_cache.shape[0], chunk, gc, max_chunks, float(scale), 1 if fused else 0, _p(fault), _s(q))
    return out


def qkv_attn_supported(nh: int, nkv: int, D: int, K: int) -> bool:
    """Whether the one-launch qkv + attention (``qkv_attn``) covers this shape: a one-row engine
    whose qkv output (nh + 2 nkv) D is under 2048 rows (the TP ranks' shards)."""
    return kernels().qkv_attn_check(nh, nkv, D, K) == 0


def qkv_attn_workspace(nh: int, nkv: int, D: int, device):
    """(granules, hctr) of ``qkv_attn``, zeroed once: the hand-off granules u64 [(nh + 2 nkv) D / 2]
    and the {exit count, hand-off epoch, o-role arrivals} counter lines int32 [3 * ATTN_CTR_PITCH]."""
    dev = torch.device(device)
    return (torch.zeros((nh + 2 * nkv) * D // 2, dtype=torch.int64, device=dev),
            torch.zeros(3 * ATTN_CTR_PITCH, dtype=torch.int32, device=dev))


QKV_ATTN_O_MAX_K = 2048  # the o-role's K (nh D) at most: 4 x 16-B chunks per lane per row


def qkv_attn_o_supported(nh: int, D: int, H: int) -> bool:
    """Whether ``qkv_attn`` can run the row's o_proj in the same launch (o-role): nh D a multiple of
    512 up to QKV_ATTN_O_MAX_K, an even number of output rows."""
    k_o = nh * D
    return k_o % 512 == 0 and k_o <= QKV_ATTN_O_MAX_K and H % 2 == 0


def qkv_attn(x, W, norm_w, eps, q_out, k_cache, v_cache, positions, slots, cos_t, sin_t, block_table, seq_len, out,
             part, counters, ws, nh, nkv, D, bs, chunk, grid_chunks, scale, fault: Optional[torch.Tensor] = None,
             w_o: Optional[torch.Tensor] = None, h: Optional[torch.Tensor] = None, add_resid: bool = True, car=None):
    """ONE row's decode qkv projection (RMSNorm prologue, RoPE + paged-KV-write epilogue, as
    ``qkv_rope``) and its attention (the fused form: ``grid_chunks`` blocks of ``chunk`` keys per kv
    head, as ``attn_decode(fused=True)``) in one launch (csrc/kernels/qkv_attn.hip): the attention
    blocks stream the cached keys' K/V under the projection and take the rotated q / the new key
    from the projection blocks as tagged granules. ``part`` / ``counters`` = ``decode_attn_workspace``
    (row 0 used), ``ws`` = ``qkv_attn_workspace``; ``fault`` as in ``attn_decode`` (4 = a lost
    hand-off granule).

    ``w_o`` / ``h`` (o-role): the token's o_proj in the same launch — ``h[0] += w_o @ out[0]``
    (``add_resid``; TP rank != 0 without ``car``: ``h[0] = w_o @ out[0]``, its all-reduce follows),
    or with ``car`` (the group's fused-all-reduce buffer) the all-reduce in the o-role's epilogue,
    rank 0 adding the residual (fault 5 = the attention output never arrived)."""
    if not x.is_cuda:
        qkv_rope(x[:1], W, norm_w, eps, q_out[:1], k_cache, v_cache, positions[:1], slots[:1], cos_t, sin_t, nh, nkv,
                 D, bs)
        out[:1].copy_(oracle.attn_decode(q_out[:1], k_cache, v_cache, block_table[:1], seq_len[:1], nh, nkv, D, bs,
                                         scale))
        if w_o is not None:
            if car is not None:
                raise ValueError("qkv_attn: the fused all-reduce runs on GPU ranks only")
            oracle.linear(out[:1], w_o, EPI_RESADD if add_resid else EPI_BF16, h[:1])
        return
    groups = counters.shape[-2] - 2
    max_chunks = part.shape[2] - groups
    if part.shape[-1] != D + 4 or counters.shape[-1] != ATTN_CTR_PITCH or grid_chunks > max_chunks:
        raise ValueError("qkv_attn: workspace does not match (decode_attn_workspace / qkv_attn_workspace)")
    gran, hctr = ws
    o_mode = 0 if w_o is None else (3 if car is not None else (1 if add_resid else 2))
    if o_mode and hctr.numel() < 3 * ATTN_CTR_PITCH:
        raise ValueError("qkv_attn: the o-role needs the 3-line counter workspace (qkv_attn_workspace)")
    bases, host, rank, world, cap = (([], 0, 0, 1, 0) if car is None else
                                     (car.bases, car.host_dev, car.rank, car.world, car.cap))
    kernels().qkv_attn(_p(x), _p(norm_w), float(eps), _p(W), x.shape[-1], _p(q_out), _p(k_cache), _p(v_cache),
                       _p(positions), _p(slots), _p(cos_t), _p(sin_t), _p(block_table), block_table.shape[-1],
                       _p(seq_len), _p(part), _p(counters), _p(out), nh, nkv, D, bs, k_cache.shape[0], chunk,
                       grid_chunks, max_chunks, float(scale), _p(fault), _p(gran), _p(hctr), o_mode, _p(w_o), _p(h),
                       0 if h is None else h.shape[-1], bases, host, rank, world, cap, _s(x))


ATTN_OPROJ_MAX_CHUNK = 512  # attn_oproj: keys per block at most (8 waves x two 32-key sub-tiles)
# kernel mode bits (A/B runs): 1 late weights; 2 the head's merger requests its own after the merge
# (1.1-1.4 us per layer faster at every length); 4 whole o_proj rows per block, no tile reduce
# (8 kv heads x 128: another 0.3-0.9 us; profiles/r4_attn_oproj_defer.md)
ATTN_OPROJ_MODE = int(os.environ.get("LLMC_ATTN_OPROJ_MODE", "7"))
# engines take the fused launch only for buckets of >= this many keys per block: below, the two
# launches measured faster (profiles/r3_attn_oproj.md: 8B at 2k keys 18.5 vs 16.3 us, at 6k-8k
# keys 18.8-21.5 vs 20.9-23.4)
ATTN_OPROJ_MIN_CHUNK = 256


def attn_oproj_min_chunk(alone: bool = False) -> int:
    """Smallest keys-per-block bucket a one-row engine runs as the fused attention + o_proj launch:
    every bucket (32) for an engine that decodes alone on its GPU (8B at 2k-5k keys: 2.84 -> 2.79,
    2.92 -> 2.85 ms/token, profiles/r5_decode_experiments.md), ATTN_OPROJ_MIN_CHUNK beside
    co-located engines (whose blocks then wait on the head merge while another engine's kernels
    want the CUs). LLMC_ATTN_OPROJ=all forces every bucket."""
    if os.environ.get("LLMC_ATTN_OPROJ") == "all" or alone:
        return 32
    return ATTN_OPROJ_MIN_CHUNK


def attn_oproj_grid(H: int, nh: int, nkv: int, D: int) -> int:
    """Blocks per kv head of the fused attention + o_proj launch (``attn_oproj``) for this shape,
    or 0 when the kernel library does not cover it: ~one block per CU over the kv heads (256 /
    nkv; Llama-3-8B: 32), each owning H / nc o_proj rows (4 o waves x 8-32 rows)."""
    top = max(1, 256 // max(1, nkv))
    # ~one block per CU; else the largest grid whose tile gives each o wave 8-32 rows
    for nc in sorted({top} | {n for n in (H // 128, H // 64, H // 32) if 0 < n <= top}, reverse=True):
        if kernels().attn_oproj_check(H, nh, nkv, D, nc, nh * D) == 0:
            return nc
    return 0


def attn_oproj_chunk(ctx_cap: int, nc: int) -> int:
    """Keys per block for a context bucket of ``ctx_cap`` keys over ``nc`` blocks per kv head (a
    multiple of 32; of 64 above 256, where each wave takes two 32-key sub-tiles), or 0 when the
    bucket needs more than ATTN_OPROJ_MAX_CHUNK keys per block."""
    per = -(-ctx_cap // nc)
    ch = max(32, (per + 31) // 32 * 32)
    if ch > 256:  # two sub-tiles per wave: 64-key units, so a wave's keys stay inside one page
        ch = (per + 63) // 64 * 64
    return ch if ch <= ATTN_OPROJ_MAX_CHUNK else 0


def attn_oproj_workspace(H: int, nh: int, nkv: int, D: int, nc: int, device):
    """(part, handoff, tile_part, counters) of ``attn_oproj``, zeroed once and never reset (the
    kernel re-arms its tickets and advances its epochs): attention partial granules f32 [nkv, nc,
    G, D/4 + 1, 4]; the merged per-head output as {bf16x2, tag} granules int32 [nkv, G D / 4, 4];
    the o_proj tile partials as {f32, tag} int64 [nc, nkv, H / nc]; counters int32 [(nkv + nc + 2)
    * 16] (head {-, epoch, ticket as u64: count + per-XCD counts}, tile tickets, {exit, tile epoch},
    {arrivals, weight-gate epoch}, one 64-B line each). The attention partials come twice ([2 nkv,
    ...]): write-through, and a copy left in the producing XCD's L2 for a same-XCD merger."""
    G = nh // nkv
    dev = torch.device(device)
    part = torch.zeros(2 * nkv, nc, G, D // 4 + 1, 4, dtype=torch.float32, device=dev)
    handoff = torch.zeros(nkv, G * D // 4, 4, dtype=torch.int32, device=dev)
    tile_part = torch.zeros(nc, nkv, H // nc, dtype=torch.int64, device=dev)
    counters = torch.zeros((nkv + nc + 2) * 16, dtype=torch.int32, device=dev)
    return part, handoff, tile_part, counters


def attn_oproj_form(H: int, nh: int, nkv: int, D: int, nc: int, chunk: int, mode: int = -1, world: int = 1) -> int:
    """The form ``attn_oproj`` takes for this shape / bucket / mode: 2 = whole o_proj rows per block
    (mode bit 2's form, the one that can run the MoE router too), 1 = tile partials, 0 = not covered."""
    return int(kernels().attn_oproj_form(H, nh, nkv, D, nc, chunk, ATTN_OPROJ_MODE if mode < 0 else mode, world))


def attn_oproj_router_workspace(nkv: int, nc: int, device):
    """(granules int64 [9, 256]: per block its 8 logit partials and sum of squares as {f32, tag};
    epoch int32 [16]) of the MoE router in ``attn_oproj(..., router=)``, zeroed once (the launch
    advances the epoch)."""
    if nkv * nc > 256:
        raise ValueError("attn_oproj router: at most 256 blocks")
    dev = torch.device(device)
    return (torch.zeros(9, 256, dtype=torch.int64, device=dev), torch.zeros(16, dtype=torch.int32, device=dev))


def attn_oproj(q, k_cache, v_cache, block_table, seq_len, w_o, h, attn_out, ws, nh, nkv, D, bs, chunk, nc, scale,
               fault: Optional[torch.Tensor] = None, stamps: Optional[torch.Tensor] = None, mode: int = -1,
               add_resid: bool = True, car=None, router=None) -> None:
    """Decode attention of ONE row followed by its o_proj and residual add, in one launch
    (csrc/kernels/attn_oproj.hip): ``h[0] += w_o @ attention(q[0])``; ``attn_out[0]`` also gets the
    attention output. ``ws`` = ``attn_oproj_workspace(...)``; ``chunk`` = ``attn_oproj_chunk(cap,
    nc)`` for a bucket whose capacity covers the sequence; ``fault`` as in ``attn_decode``;
    ``stamps`` (diagnostics): int64 [nkv, nc, 8] per-block phase times (see the kernel's host
    function); ``mode`` bit 0: o_proj weights requested after the head ticket, bit 1 (with bit 0):
    the head's merger requests its own after the merge, bit 2 (with bit 0; 8 kv heads, G = 4, D =
    128, 128-row tiles, else ignored): whole o_proj rows per block (-1 = ATTN_OPROJ_MODE).

    Tensor-parallel ranks (``h`` gets this rank's row-parallel share): ``add_resid`` False writes
    h = W_o . attention (a rank != 0 whose all-reduce follows as its own launch); ``car`` (the
    group's fused-all-reduce ``CustomAllReduce``) runs the all-reduce in the kernel's tile-reducer
    epilogue: h = the sum over ranks, rank 0's term carrying the residual (pass add_resid = rank 0).

    ``router`` = (norm_w, W_router, eps, k, w_out, ids_out, rws): the MoE layer's decode router on
    the launch's output row in the same launch — ``moe_router(h, norm_w, eps, W_router, k, w_out,
    ids_out)``'s outputs up to the logits' summation order; ``rws`` =
    ``attn_oproj_router_workspace``; needs ``attn_oproj_form(...) == 2``, no ``car`` and an engine
    alone on its GPU (block 0 of the grid waits on the others' router partials; GPU only)."""
    H = h.shape[-1]
    if not q.is_cuda:
        if car is not None:
            raise ValueError("attn_oproj: the fused all-reduce runs on GPU ranks only")
        a = oracle.attn_decode(q[:1], k_cache, v_cache, block_table[:1], seq_len[:1], nh, nkv, D, bs, scale)
        attn_out[:1].copy_(a)
        oracle.linear(attn_out[:1], w_o, EPI_RESADD if add_resid else EPI_BF16, h[:1])
        if router is not None:
            raise ValueError("attn_oproj: the router partials are a GPU form")
        return
    if chunk <= 0 or chunk * nc < 1 or nc != ws[0].shape[1]:
        raise ValueError("attn_oproj: chunk / workspace do not match (attn_oproj_chunk, attn_oproj_workspace)")
    part, handoff, tile_part, counters = ws
    bases, host, rank, world, cap = (([], 0, 0, 1, 0) if car is None else
                                     (car.bases, car.host_dev, car.rank, car.world, car.cap))
    rt = (None, None, 0.0, 0, 0, None, None, None, None)
    if router is not None:
        if car is not None:
            raise ValueError("attn_oproj: the fused router runs on one-GPU engines only")
        norm_w, W_r, eps, k, w_out, ids_out, (rpart, repoch) = router
        if tuple(rpart.shape) != (9, 256) or W_r.shape[1] != H:
            raise ValueError("attn_oproj: router workspace / weights do not match")
        rt = (norm_w, W_r, float(eps), W_r.shape[0], int(k), w_out, ids_out, rpart, repoch)
    kernels().attn_oproj(_p(q), _p(k_cache), _p(v_cache), _p(block_table), block_table.shape[-1], _p(seq_len), _p(w_o),
                         _p(h), _p(attn_out), _p(part), _p(handoff), _p(tile_part), _p(counters), _p(fault), H, nh, nkv,
                         D, bs, k_cache.shape[0], chunk, nc, float(scale),
                         ATTN_OPROJ_MODE if mode < 0 else mode, _p(stamps), int(bool(add_resid)), bases, host, rank,
                         world, cap, _p(rt[0]), _p(rt[1]), rt[2], rt[3], rt[4], _p(rt[5]), _p(rt[6]), _p(rt[7]),
                         _p(rt[8]), _s(h))


# KV split of the prefill attention: -1 = the kernel library's plan (llmc_attn_prefill_plan),
# 1 = never, N = split every group of >= 2 * LLMC_PREFILL_KMIN (default 8) key tiles up to N ways
PREFILL_KSPLIT = int(os.environ.get("LLMC_PREFILL_KSPLIT", "-1"))
PREFILL_KMIN = int(os.environ.get("LLMC_PREFILL_KMIN", "8"))


def attn_prefill_plan(B, max_qlen, max_ctx, nh, nkv, ksplit=None, kmin=None, D=128, bs=64):
    """(ksplit, kmin) of a prefill attention launch (csrc/kernels/attn_prefill.hip): row-tile groups
    of >= 2 kmin key tiles run on min(ksplit, tiles // kmin) blocks; (1, _) = no split. ``D`` / ``bs``
    (head dim, KV page size) tell the plan which unsplit block forms it competes against."""
    k = PREFILL_KSPLIT if ksplit is None else int(ksplit)
    if k < 0:
        return tuple(kernels().attn_prefill_plan(B, int(max_qlen), int(max_ctx), nh, nkv, int(D), int(bs)))
    return max(1, min(k, 4)), int(PREFILL_KMIN if kmin is None else kmin)


def attn_prefill_counters(B, max_qlen, nh, nkv) -> int:
    """Arrival counters of a split prefill launch: one per (sequence, row-tile group of the 8-wave
    split grid, kv head) — the kernel library's own count (``llmc_attn_prefill_counters``), used by
    both the workspace allocator and ``attn_prefill``'s reuse check."""
    return int(kernels().attn_prefill_counters(int(B), int(max_qlen), int(nh), int(nkv)))


def attn_prefill_workspace(ksplit, T, nh, D, device, B=1, nkv=1, max_qlen=None):
    """A split prefill's hand-off state: f32 partials ([ksplit][T][nh][D] O, then [ksplit][T][nh][2]
    (m, l)) and zeroed arrival counters (one per (sequence, row-tile group, kv head), re-armed by the
    kernel, so one workspace serves every layer of a prefill on one stream)."""
    return (torch.empty(ksplit * T * nh * (D + 2), dtype=torch.float32, device=device),
            torch.zeros(max(1, attn_prefill_counters(B, max_qlen or T, nh, nkv)), dtype=torch.int32, device=device))


def attn_prefill(q, k_cache, v_cache, block_tables, q_start, q_lens, ctx_lens, out, max_qlen, nh, nkv, D, bs, scale,
                 max_ctx=None, ksplit=None, kmin=None, ws=None, form=None):
    """Causal paged prefill attention. ``max_ctx`` (default ``max_qlen``) feeds the KV-split plan;
    ``ksplit``/``kmin`` override it; ``ws`` is a caller-held attn_prefill_workspace reused across
    layers (it must not be shared by launches that can run concurrently); ``form`` forces the block
    form of an unsplit launch (0 = 8 waves, 1 = paired row tiles, 2 = 4 waves, 3 = key halves;
    default: the kernel library's choice, ``kernels().attn_prefill_form``)."""
    if not q.is_cuda:
        return oracle.attn_prefill(q, k_cache, v_cache, block_tables, q_start, q_lens, ctx_lens, nh, nkv, D, bs,
                                   scale, out)
    B = q_lens.shape[0]
    T = q.shape[0]
    k, km = attn_prefill_plan(B, max_qlen, max_qlen if max_ctx is None else max_ctx, nh, nkv, ksplit, kmin, D, bs)
    part = ctr = 0
    if k > 1:
        need_c = attn_prefill_counters(B, max_qlen, nh, nkv)
        if ws is None or ws[0].numel() < k * T * nh * (D + 2) or ws[1].numel() < need_c:
            ws = attn_prefill_workspace(k, T, nh, D, q.device, B, nkv, max_qlen)
        part, ctr = _p(ws[0]), _p(ws[1])
    try:
        kernels().attn_prefill(_p(q), q.stride(0), _p(k_cache), _p(v_cache), _p(block_tables), block_tables.stride(0),
                               _p(q_start), _p(q_lens), _p(ctx_lens), _p(out), out.stride(0), B, int(max_qlen), nh,
                               nkv, D, bs, float(scale), k, km, part, ctr, T, -1 if form is None else int(form), _s(q))
    except Exception:
        # a failed launch may leave arrival counters armed; the next launch on this workspace
        # would merge before its partials arrived: re-zero them (stream-ordered)
        if k > 1:
            ws[1].zero_()
        raise
    return out


def sample_parts() -> int:
    return kernels().sample_parts()


def sample(logits, inv_temp, top_k, top_p, seeds, positions, next_tok, workspace_v=None, workspace_i=None,
           tokens_in=None, seq_lens=None, slots=None, block_tables=None, bs=0, out_tokens=None, out_count=None,
           use_topkp: bool = False):
    """Sample one token per row and (optionally) advance the device decode state in the same launch."""
    if not logits.is_cuda:
        tok = oracle.sample(logits, inv_temp, top_k, top_p, seeds, positions)
        next_tok.copy_(tok)
        _advance_cpu(tok, tokens_in, positions, seq_lens, slots, block_tables, bs, out_tokens, out_count)
        return next_tok
    B, V = logits.shape
    cap = out_tokens.shape[1] if out_tokens is not None else 0
    kernels().sample(_p(logits), logits.stride(0), B, V, _p(inv_temp), _p(top_k), _p(top_p), _p(seeds), _p(positions),
                     _p(workspace_v), _p(workspace_i), _p(next_tok), _p(tokens_in), _p(seq_lens), _p(slots),
                     _p(block_tables), block_tables.stride(0) if block_tables is not None else 0, bs, _p(out_tokens),
                     _p(out_count), cap, 1 if use_topkp else 0, _s(logits))
    return next_tok


def _advance_cpu(tok, tokens_in, positions, seq_lens, slots, block_tables, bs, out_tokens, out_count):
    if tokens_in is None:
        return
    B = tok.shape[0]
    for b in range(B):
        t = int(tok[b])
        if out_tokens is not None:
            c = int(out_count[b])
            if c < out_tokens.shape[1]:
                out_tokens[b, c] = t
            out_count[b] = c + 1
        if tokens_in is not None:
            tokens_in[b] = t
        if positions is not None:
            p = int(positions[b]) + 1
            positions[b] = p
            if seq_lens is not None:
                seq_lens[b] = p + 1
            if slots is not None and block_tables is not None:
                slots[b] = int(block_tables[b, p // bs]) * bs + p % bs


# -- MoE -----------------------------------------------------------------------------------------
MOE_TILE = 128       # row tile of the small-group grouped GEMM (128 x 128 kernel)
MOE_TILE_LARGE = 256  # ... and of the 256 x 256 LDS-DMA pipeline


def moe_tile(npairs: int, E: int) -> int:
    """Row tile of the grouped expert GEMM: the 256 x 256 pipeline once the (token, slot) pairs
    average >= 256 rows per expert (padding stays < 1/2 tile per expert), else 128-row tiles."""
    return MOE_TILE_LARGE if npairs >= MOE_TILE_LARGE * E else MOE_TILE


def moe_route(logits: torch.Tensor, k: int, w_out: torch.Tensor, ids_out: torch.Tensor):
    if not logits.is_cuda:
        w, ids = oracle.moe_route(logits, k)
        w_out.copy_(w)
        ids_out.copy_(ids)
        return w_out, ids_out
    T, E = logits.shape
    kernels().moe_route(_p(logits), T, E, k, _p(w_out), _p(ids_out), _s(logits))
    return w_out, ids_out


def moe_route_fused(x: torch.Tensor, W_router: torch.Tensor, k: int, w_out: torch.Tensor, ids_out: torch.Tensor):
    """Prefill router in one launch: logits = x . W_router^T (f32), softmax top-k, renormalised
    (K9; csrc/kernels/moe.hip moe_route_fused_kernel). x [T, H] bf16 (normalised rows), W_router
    [E <= 16, H]."""
    if not x.is_cuda:
        return moe_route(oracle.linear(x, W_router, EPI_F32), k, w_out, ids_out)
    T, H = x.shape
    kernels().moe_route_fused(_p(x), x.stride(0), _p(W_router), T, W_router.shape[0], H, k, _p(w_out), _p(ids_out),
                              _s(x))
    return w_out, ids_out


def moe_route_fused_supported(E: int, H: int) -> bool:
    return E <= 16 and H % 8 == 0 and H <= 8192 and E * H * 2 <= 160 * 1024


def moe_max_tiles(npairs: int, E: int, tile: int = MOE_TILE) -> int:
    return (npairs + tile - 1) // tile + E


def moe_align(ids: torch.Tensor, E: int, sorted_rows, tile_expert, tile_count, counts=None, tile: int = MOE_TILE):
    T, k = ids.shape
    kernels().moe_align(_p(ids), T, k, E, tile, _p(sorted_rows), _p(tile_expert), _p(tile_count), _p(counts),
                        _s(ids))


def moe_gemm(A, W_experts, sorted_rows, tile_expert, tile_count, out, N, K, max_tiles, a_row_div, epi=EPI_BF16,
             tile: int = MOE_TILE):
    """Grouped expert GEMM (K11) over moe_align's list (same ``tile``): out[sorted_rows[i]] =
    epi(A[sorted_rows[i] // a_row_div] . W[tile_expert[i // tile]]^T); EPI_SILU writes silu(gate) *
    up of the interleaved gate/up columns ([., N / 2])."""
    kernels().moe_gemm(_p(A), A.stride(0), A.shape[0], _p(W_experts), _p(sorted_rows), _p(tile_expert),
                       _p(tile_count), _p(out), out.stride(0), N, K, max_tiles, a_row_div, epi, tile, _s(A))
    return out


def moe_combine(y, w, ids, h, rows: Optional[torch.Tensor] = None):
    """h[t] += sum_j w[t, j] * y[t*k + j] (K12; fixed order, f32, zero-weight pairs skipped);
    ``rows`` [T*k] int32: pair (t, j)'s result is y row rows[t*k + j] instead (the slots of the
    expert-parallel all-to-all, ``moe_ep_dispatch``)."""
    if not h.is_cuda:
        if rows is not None:
            y = y.index_select(0, rows.long().clamp(min=0))
        return oracle.moe_combine(y, w, h)
    T, k = w.shape
    kernels().moe_combine(_p(y), _p(w), _p(rows), _p(h), T, k, h.shape[1], _s(h))
    return h


def moe_ep_dispatch(ids: torch.Tensor, n_local: int, n_ranks: int, cap: int):
    """Expert-parallel all-to-all plan of a token shard's (token, slot) pairs (C4), on the device:
    pair i goes to rank d = ids[i] // n_local, slot d * cap + (its rank among d's pairs, in pair
    order). -> (send_pair [n*cap] i32 pair index or -1, send_e [n*cap] i32 expert id local to d or
    -1, pair_slot [T*k] i32, counts [n] i32). ``cap`` >= T*k (every pair may pick one rank)."""
    P = ids.numel()
    dev = ids.device
    i32 = dict(dtype=torch.int32, device=dev)
    send_pair = torch.empty(n_ranks * cap, **i32)
    send_e = torch.empty(n_ranks * cap, **i32)
    slot = torch.empty(P, **i32)
    counts = torch.empty(n_ranks, **i32)
    if not ids.is_cuda:
        sp, se, sl, cn = oracle.moe_ep_dispatch(ids, n_local, n_ranks, cap)
        return send_pair.copy_(sp), send_e.copy_(se), slot.copy_(sl), counts.copy_(cn)
    kernels().moe_ep_dispatch(_p(ids), P, int(n_local), int(n_ranks), int(cap), _p(send_pair), _p(send_e), _p(slot),
                              _p(counts), _s(ids))
    return send_pair, send_e, slot, counts


def gather_rows(x: torch.Tensor, rows: torch.Tensor, div: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[j] = x[rows[j] // div], zero rows where rows[j] < 0 (the expert-parallel send buffer)."""
    M = rows.numel()
    if out is None:
        out = torch.empty(M, x.shape[1], dtype=x.dtype, device=x.device)
    if not x.is_cuda:
        r = rows.long()
        out.copy_(torch.where((r >= 0).unsqueeze(1), x.index_select(0, (r.clamp(min=0) // div)),
                              torch.zeros((), dtype=x.dtype)))
        return out
    _bf16(x, "gather_rows.x")
    kernels().gather_rows(_p(x), x.stride(0), _p(rows), M, int(div), x.shape[1], _p(out), out.stride(0), _s(x))
    return out


def moe_gemv(x, W_experts, ids, x_div, out, N, K, epi, norm_w=None, eps: float = 1e-5):
    """Decode expert GEMV over (token, slot) pairs; ``norm_w``: RMS-normalise x (raw hidden rows)
    in the prologue."""
    npairs = ids.numel()
    kernels().moe_gemv(npairs, _p(x), x.stride(0), _p(norm_w) if norm_w is not None else 0, float(eps),
                       _p(W_experts), _p(ids), x_div, _p(out), out.stride(0), N, K, epi, _s(x))
    return out


def moe_gemvm(x, W_experts, ids, x_div, out, N, K, epi, norm_w=None, eps: float = 1e-5):
    """Batched MoE decode (<= MOE_GEMVM_MAX_TOKENS tokens) on the MFMA form with the pairs grouped by expert: every
    routed expert's weights stream once for all its pairs (``moe_gemv`` streams them once per pair).
    out[p] = W[ids[p]] . x[p // x_div]; pairs with id -1 (another rank's expert) are not written."""
    if not x.is_cuda:
        raise ValueError("moe_gemvm: GPU only (the CPU path is moe_gemv's oracle)")
    P, E = ids.numel(), W_experts.shape[0]
    if ids.dim() != 2 or ids.shape[0] > MOE_GEMVM_MAX_TOKENS:
        raise ValueError(f"moe_gemvm: ids [tokens <= {MOE_GEMVM_MAX_TOKENS}, k], got {tuple(ids.shape)}")
    kernels().moe_gemvm(P, _p(x), x.stride(0), _p(norm_w) if norm_w is not None else 0, float(eps), _p(W_experts),
                        _p(ids), x_div, E, _p(out), out.stride(0), N, K, epi, _s(x))
    return out


def moe_down_combine(act, W_down, ids, w, h, N, K):
    """Decode MoE down projection fused with the combine (top-2): h[t] += sum_j w[t, j] *
    (W_down[ids[t, j]] . act[t*2 + j]), fixed order, f32."""
    T, k = ids.shape
    kernels().moe_down_combine(T, _p(act), act.stride(0), _p(W_down), _p(ids), _p(w), _p(h), h.stride(0), N, K, k,
                               _s(act))
    return h


def moe_router(x, norm_w, eps: float, W_router, k: int, w_out, ids_out):
    """Decode router, one launch: rmsnorm(x) * norm_w -> router logits -> softmax top-k (renormalised).
    x [T, H] bf16 (raw hidden rows), W_router [E, H]."""
    if not x.is_cuda:
        xn = oracle.rmsnorm(x, norm_w, eps)
        logits = oracle.linear(xn, W_router, EPI_F32)
        return moe_route(logits, k, w_out, ids_out)
    T, H = x.shape
    E = W_router.shape[0]
    kernels().moe_router(_p(x), x.stride(0), _p(norm_w), float(eps), _p(W_router), T, E, H, k, _p(w_out), _p(ids_out),
                         _s(x))
    return w_out, ids_out


def moe_ep_localize(ids, w, e0: int, n_local: int, lids_out, lw_out):
    """Expert parallel: global expert ids -> local ids of experts [e0, e0 + n_local) on this rank,
    -1 (and weight 0) for the others; device-side, so the decode graph stays replayable."""
    if not ids.is_cuda:
        lids, lw = oracle.moe_ep_localize(ids, w, e0, n_local)
        lids_out.copy_(lids)
        lw_out.copy_(lw)
        return lids_out, lw_out
    kernels().moe_ep_localize(_p(ids), _p(w), ids.numel(), int(e0), int(n_local), _p(lids_out), _p(lw_out), _s(ids))
    return lids_out, lw_out
