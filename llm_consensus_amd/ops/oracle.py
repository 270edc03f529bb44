"""PyTorch reference semantics of every HIP kernel (test oracles + CPU execution of model logic).

These define the numerics the kernels implement (f32 math, bf16 rounding points). CUDA tensors
NEVER route here — ``ops/__init__.py`` sends them to the HIP module and raises if it is missing;
CPU tensors use these so the model / TP / engine logic is testable on the CPU-only runner.
"""

from __future__ import annotations

import math
from typing import Optional

import torch

EPI_BF16, EPI_F32, EPI_RESADD, EPI_SILU, EPI_ROPE = 0, 1, 2, 3, 4


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * inv * w.float()).to(torch.bfloat16)


def embedding(ids: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    return table[ids.long().clamp(0, table.shape[0] - 1)]


def silu_mul_interleaved(gu: torch.Tensor) -> torch.Tensor:
    g = gu[..., 0::2].float()
    u = gu[..., 1::2].float()
    return (torch.nn.functional.silu(g) * u).to(torch.bfloat16)


def linear(x: torch.Tensor, W: torch.Tensor, epi: int, out: Optional[torch.Tensor] = None,
           norm_w: Optional[torch.Tensor] = None, eps: float = 1e-5) -> torch.Tensor:
    if epi == EPI_ROPE:
        raise ValueError("EPI_ROPE: use qkv_rope")
    if norm_w is not None:
        x = rmsnorm(x, norm_w, eps)
    acc = x.float() @ W.float().t()
    if epi == EPI_BF16:
        res = acc.to(torch.bfloat16)
    elif epi == EPI_F32:
        res = acc
    elif epi == EPI_RESADD:
        assert out is not None
        res = (out.float() + acc).to(torch.bfloat16)
    elif epi == EPI_SILU:
        res = (torch.nn.functional.silu(acc[..., 0::2]) * acc[..., 1::2]).to(torch.bfloat16)
    else:
        raise ValueError(epi)
    if out is not None:
        out.copy_(res)
        return out
    return res


def rope_tables(inv_freq, max_pos: int):
    inv = torch.tensor(inv_freq, dtype=torch.float64)
    t = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return torch.cos(ang).float(), torch.sin(ang).float()


def rope_kv_write(qkv, positions, cos_t, sin_t, k_cache, v_cache, slots, nh, nkv, D, bs, q_out):
    """qkv rows hold Q and K heads PAIR-INTERLEAVED ([x0, x_h, x1, x_{h+1}, ...], h = D/2);
    rotated Q goes to ``q_out`` [T, nh*D] in canonical order, rotated K / raw V to the cache."""
    T = qkv.shape[0]
    half = D // 2
    pos = positions.long()
    c = cos_t[pos].unsqueeze(1)  # [T,1,half]
    s = sin_t[pos].unsqueeze(1)
    qk = qkv[:, : (nh + nkv) * D].view(T, nh + nkv, half, 2).float()
    x1, x2 = qk[..., 0], qk[..., 1]
    rot = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(torch.bfloat16)
    q_out[:, : nh * D] = rot[:, :nh].reshape(T, nh * D)
    if slots is not None:
        v = qkv[:, (nh + nkv) * D:(nh + 2 * nkv) * D].view(T, nkv, D)
        for t in range(T):
            sl = int(slots[t])
            if sl < 0:
                continue
            page, off = sl // bs, sl % bs
            k_cache[page, :, off] = rot[t, nh:]
            v_cache[page, :, off] = v[t]


def _gather_kv(cache, bt_row, L, bs):
    """[L, nkv, D] from a paged cache [nb, nkv, bs, D]."""
    idx = torch.arange(L, device=cache.device)
    pages = bt_row.to(cache.device)[(idx // bs)].long()
    return cache[pages, :, (idx % bs)]


def attn_decode(q, k_cache, v_cache, block_tables, seq_lens, nh, nkv, D, bs, scale):
    B = q.shape[0]
    G = nh // nkv
    out = torch.empty(B, nh * D, dtype=torch.bfloat16)
    for b in range(B):
        L = int(seq_lens[b])
        k = _gather_kv(k_cache, block_tables[b], L, bs).float()  # [L, nkv, D]
        v = _gather_kv(v_cache, block_tables[b], L, bs).float()
        qb = q[b, : nh * D].view(nh, D).float()
        kk = k.repeat_interleave(G, dim=1)  # [L, nh, D]
        vv = v.repeat_interleave(G, dim=1)
        s = torch.einsum("hd,lhd->hl", qb, kk) * scale
        p = torch.softmax(s, dim=-1)
        out[b] = torch.einsum("hl,lhd->hd", p, vv).reshape(-1).to(torch.bfloat16)
    return out


def attn_prefill(q, k_cache, v_cache, block_tables, q_start, q_lens, ctx_lens, nh, nkv, D, bs, scale, out):
    G = nh // nkv
    for b in range(len(q_lens)):
        ql, ctx, q0 = int(q_lens[b]), int(ctx_lens[b]), int(q_start[b])
        if ql == 0:
            continue
        k = _gather_kv(k_cache, block_tables[b], ctx, bs).float().repeat_interleave(G, dim=1)
        v = _gather_kv(v_cache, block_tables[b], ctx, bs).float().repeat_interleave(G, dim=1)
        qb = q[q0:q0 + ql, : nh * D].view(ql, nh, D).float()
        s = torch.einsum("qhd,khd->hqk", qb, k) * scale
        qpos = torch.arange(ctx - ql, ctx, device=s.device).view(1, ql, 1)
        kpos = torch.arange(ctx, device=s.device).view(1, 1, ctx)
        s = s.masked_fill(kpos > qpos, float("-inf"))
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("hqk,khd->qhd", p, v)
        out[q0:q0 + ql, : nh * D] = o.reshape(ql, nh * D).to(torch.bfloat16)
    return out


# -- sampler ------------------------------------------------------------------------------------
_M0, _M1, _W0, _W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
_MASK = 0xFFFFFFFF


def philox_draw(key: int, idx: torch.Tensor, step: int) -> torch.Tensor:
    """Vectorised Philox4x32-10, identical to the device version (returns word 0)."""
    c0 = idx.to(torch.int64) & _MASK
    c1 = torch.full_like(c0, step & _MASK)
    c2 = torch.full_like(c0, 0x5EED)
    c3 = torch.zeros_like(c0)
    k0, k1 = key & _MASK, (key >> 32) & _MASK
    for _ in range(10):
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = (p0 >> 32) & _MASK, p0 & _MASK
        hi1, lo1 = (p1 >> 32) & _MASK, p1 & _MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & _MASK, lo1, (hi0 ^ c3 ^ k1) & _MASK, lo0
        k0 = (k0 + _W0) & _MASK
        k1 = (k1 + _W1) & _MASK
    return c0


def gumbel(key: int, idx: torch.Tensor, step: int) -> torch.Tensor:
    r = philox_draw(key, idx, step)
    u = ((r >> 8).float() + 0.5) * (1.0 / 16777216.0)
    return -torch.log(-torch.log(u))


def sample(logits: torch.Tensor, inv_temp, top_k, top_p, seeds, positions) -> torch.Tensor:
    """Reference sampler: greedy if inv_temp <= 0; else Gumbel-max over the top-k/top-p set."""
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.int32)
    idx = torch.arange(V)
    for b in range(B):
        row = logits[b].float()
        it = float(inv_temp[b])
        k = int(top_k[b]) if top_k is not None else 0
        p = float(top_p[b]) if top_p is not None else 1.0
        keep = torch.ones(V, dtype=torch.bool)
        if k > 0 and k < V:
            kth = torch.topk(row, k).values[-1]
            keep &= row >= kth
        if it > 0 and p < 1.0:
            m = row.max()
            w = torch.exp((row - m) * it) * keep
            z = w.sum()
            order = torch.argsort(row, descending=True, stable=True)
            cum = torch.cumsum(w[order], 0)
            cut = int(torch.searchsorted(cum, p * z).item())
            cut = min(cut, V - 1)
            thr = row[order[cut]]
            keep &= row >= thr
        if it <= 0:
            v = torch.where(keep, row, torch.tensor(float("-inf")))
        else:
            g = gumbel(int(seeds[b]), idx, int(positions[b]))
            v = torch.where(keep, row * it + g, torch.tensor(float("-inf")))
        mx = v.max()
        out[b] = int(torch.nonzero(v == mx)[0].item())
    return out


# -- MoE ------------------------------------------------------------------------------------------
def moe_route(logits: torch.Tensor, k: int):
    p = torch.softmax(logits.float(), dim=-1)
    w, ids = torch.topk(p, k, dim=-1)
    w = w / w.sum(-1, keepdim=True)
    return w, ids.to(torch.int32)


def moe_ffn(x: torch.Tensor, w_gu: torch.Tensor, w_down: torch.Tensor, rw: torch.Tensor, ids: torch.Tensor,
            h: torch.Tensor) -> torch.Tensor:
    """h += sum_j rw[t,j] * down_e(silu_mul(gate_up_e(x_t))) with per-pair bf16 rounding of the
    intermediate tensors exactly where the kernels round."""
    T, k = ids.shape
    y = torch.empty(T * k, h.shape[1], dtype=torch.bfloat16)
    for t in range(T):
        for j in range(k):
            e = int(ids[t, j])
            gu = (x[t:t + 1].float() @ w_gu[e].float().t()).to(torch.bfloat16)
            act = silu_mul_interleaved(gu)
            y[t * k + j] = (act.float() @ w_down[e].float().t()).to(torch.bfloat16)[0]
    yk = y.view(T, k, -1).float()
    s = (rw.float().unsqueeze(-1) * yk).sum(1)
    h.copy_((h.float() + s).to(torch.bfloat16))
    return h


def moe_combine(y: torch.Tensor, w: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    """h[t] += sum_j w[t,j] * y[t*k + j] in f32 (pairs with weight 0 — other ranks' experts
    under expert parallelism — are skipped, their y rows may be garbage)."""
    T, k = w.shape
    yk = y.view(T, k, -1).float()
    wf = w.float().unsqueeze(-1)
    s = torch.where(wf != 0, wf * yk, torch.zeros((), dtype=torch.float32)).sum(1)
    h.copy_((h.float() + s).to(torch.bfloat16))
    return h


def moe_ep_localize(ids: torch.Tensor, w: torch.Tensor, e0: int, n_local: int):
    """Global expert ids -> this rank's local ids (-1 = another rank's expert, weight 0)."""
    loc = (ids >= e0) & (ids < e0 + n_local)
    lids = torch.where(loc, ids - e0, torch.full_like(ids, -1))
    lw = torch.where(loc, w, torch.zeros_like(w))
    return lids.to(torch.int32), lw


def moe_ep_dispatch(ids: torch.Tensor, n_local: int, n_ranks: int, cap: int):
    """Reference of the expert-parallel dispatch plan (see ops.moe_ep_dispatch): stable slots per
    destination rank in pair order, -1 padding."""
    flat = ids.reshape(-1).long()
    send_pair = torch.full((n_ranks * cap,), -1, dtype=torch.int32)
    send_e = torch.full((n_ranks * cap,), -1, dtype=torch.int32)
    slot = torch.empty(flat.numel(), dtype=torch.int32)
    counts = torch.zeros(n_ranks, dtype=torch.int32)
    for i, e in enumerate(flat.tolist()):
        d = e // n_local
        s = d * cap + int(counts[d])
        counts[d] += 1
        send_pair[s], send_e[s], slot[i] = i, e - d * n_local, s
    return send_pair, send_e, slot, counts


def softmax_scale(D: int) -> float:
    return 1.0 / math.sqrt(D)


# -- whole-model reference forward (tests) ------------------------------------------------------
@torch.no_grad()
def reference_logits(w, cfg, ids, out_pos, cos_t: torch.Tensor, sin_t: torch.Tensor, chunk: int = 1024,
                     attn_chunk: int = 512, p_bf16: bool = False) -> torch.Tensor:
    """fp32 PyTorch forward of a ``TransformerWeights`` model (one TP=1 model or one rank's shard
    standing alone) over the token sequence ``ids``: the last-layer logits [len(out_pos), V_local]
    f32 at positions ``out_pos``. Every matmul, norm, RoPE, softmax and SiLU is fp32; activations
    are rounded to bf16 exactly where the engine stores them (normed rows, q/k/v, attention
    output, residual stream, SiLU product, expert outputs), so it is the engine's semantics at
    full precision — the oracle of the full-depth teacher-forced decode tests. Runs on the
    weights' device (the GPU for full-size models: fp32 copies are made one weight at a time),
    in ``chunk``-token slices for the projections and ``attn_chunk``-query slices for causal
    attention over the whole sequence. ``p_bf16``: round the attention probabilities to bf16
    before the P.V product, as the MFMA attention kernels do (their row sums stay f32)."""
    dev = w.embed.device
    bf, f32 = torch.bfloat16, torch.float32
    T = len(ids)
    nh, nkv, D = w.nh, w.nkv, cfg.head_dim
    G, half = nh // nkv, D // 2
    idx = torch.as_tensor(ids, dtype=torch.long, device=dev)
    pos = torch.arange(T, device=dev)
    cos, sin = cos_t.to(dev)[pos].unsqueeze(1), sin_t.to(dev)[pos].unsqueeze(1)  # [T, 1, half]
    h = w.embed[idx.clamp(0, w.embed.shape[0] - 1)].clone()
    scale = 1.0 / math.sqrt(D)

    def lin(x, W):  # fp32 x @ W^T in token slices -> fp32
        Wf = W.float()
        return torch.cat([x[i:i + chunk].float() @ Wf.t() for i in range(0, x.shape[0], chunk)])

    for L in w.layers:
        xn = rmsnorm(h, L.ln1, cfg.rms_eps)
        qkv = lin(xn, L.w_qkv).to(bf)
        qk = qkv[:, : (nh + nkv) * D].view(T, nh + nkv, half, 2).float()
        x1, x2 = qk[..., 0], qk[..., 1]
        rot = torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(bf)  # [T, nh + nkv, D]
        q, k = rot[:, :nh].float(), rot[:, nh:].float()
        v = qkv[:, (nh + nkv) * D:(nh + 2 * nkv) * D].view(T, nkv, D).float()
        attn = torch.empty(T, nh * D, dtype=bf, device=dev)
        for q0 in range(0, T, attn_chunk):
            q1 = min(T, q0 + attn_chunk)
            qc = q[q0:q1].view(q1 - q0, nkv, G, D)                        # [q, kv, G, D]
            s = torch.einsum("qkgd,tkd->kgqt", qc, k[:q1]) * scale         # keys 0..q1-1
            mask = torch.arange(q1, device=dev).view(1, -1) > torch.arange(q0, q1, device=dev).view(-1, 1)
            s.masked_fill_(mask, float("-inf"))
            if p_bf16:
                e = torch.exp(s - s.amax(-1, keepdim=True))
                o = torch.einsum("kgqt,tkd->qkgd", e.to(bf).float(), v[:q1]) / e.sum(-1).permute(2, 0, 1).unsqueeze(-1)
                del e
            else:
                p = torch.softmax(s, dim=-1)
                o = torch.einsum("kgqt,tkd->qkgd", p, v[:q1])
                del p
            attn[q0:q1] = o.reshape(q1 - q0, nh * D).to(bf)
            del s, o
        h = (h.float() + lin(attn, L.w_o)).to(bf)
        xn = rmsnorm(h, L.ln2, cfg.rms_eps)
        if cfg.is_moe:
            rw, rid = moe_route(lin(xn, L.w_router), cfg.top_k_experts)
            k_ = cfg.top_k_experts
            y = torch.zeros(T * k_, cfg.hidden, dtype=bf, device=dev)
            flat = rid.view(-1).long()
            for e in range(L.w_gu.shape[0]):
                sel = (flat == e).nonzero().view(-1)
                if sel.numel() == 0:
                    continue
                xe = xn[sel // k_]
                gu = lin(xe, L.w_gu[e])
                act = (torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]).to(bf)
                y[sel] = lin(act, L.w_down[e]).to(bf)
            s = (rw.float().unsqueeze(-1) * y.view(T, k_, -1).float()).sum(1)
            h = (h.float() + s).to(bf)
        else:
            gu = lin(xn, L.w_gu)
            act = (torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]).to(bf)
            del gu
            h = (h.float() + lin(act, L.w_down)).to(bf)
    sel = torch.as_tensor(out_pos, dtype=torch.long, device=dev)
    hn = rmsnorm(h[sel], w.final_norm, cfg.rms_eps)
    return hn.float() @ w.lm_head.float().t()


@torch.no_grad()
def reference_decode_layer(L, cfg, h_in: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                           bt_row: torch.Tensor, pos: int, cos_t: torch.Tensor, sin_t: torch.Tensor, nh: int, nkv: int,
                           bs: int, p_bf16: bool = False) -> torch.Tensor:
    """fp32 reference of ONE dense decode layer for one token at position ``pos``, fed the engine's
    own layer input ``h_in`` [1, H] and the engine's own paged K/V of positions [0, pos) (the
    token's own k/v are computed here): the layer output h [1, H] bf16, rounded where the engine
    rounds (normed rows, q/k/v, attention output, residual stream, SiLU product). Isolates one
    layer's error from the depth amplification of a whole-model comparison."""
    dev = h_in.device
    bf = torch.bfloat16
    D = cfg.head_dim
    G, half = nh // nkv, D // 2
    xn = rmsnorm(h_in, L.ln1, cfg.rms_eps)
    qkv = (xn.float() @ L.w_qkv.float().t()).to(bf)[0]
    qk = qkv[: (nh + nkv) * D].view(nh + nkv, half, 2).float()
    c, sn = cos_t.to(dev)[pos].float(), sin_t.to(dev)[pos].float()
    x1, x2 = qk[..., 0], qk[..., 1]
    rot = torch.cat([x1 * c - x2 * sn, x2 * c + x1 * sn], dim=-1).to(bf)  # [nh + nkv, D]
    q = rot[:nh].float().view(nkv, G, D)
    k_new = rot[nh:].float()
    v_new = qkv[(nh + nkv) * D:(nh + 2 * nkv) * D].view(nkv, D).float()
    k_old = _gather_kv(k_cache, bt_row, pos, bs).float()  # [pos, nkv, D]
    v_old = _gather_kv(v_cache, bt_row, pos, bs).float()
    k = torch.cat([k_old, k_new.unsqueeze(0)])
    v = torch.cat([v_old, v_new.unsqueeze(0)])
    s = torch.einsum("kgd,tkd->kgt", q, k) / math.sqrt(D)
    if p_bf16:
        e = torch.exp(s - s.amax(-1, keepdim=True))
        o = torch.einsum("kgt,tkd->kgd", e.to(bf).float(), v) / e.sum(-1, keepdim=True)
    else:
        o = torch.einsum("kgt,tkd->kgd", torch.softmax(s, dim=-1), v)
    attn = o.reshape(1, nh * D).to(bf)
    h = (h_in.float() + attn.float() @ L.w_o.float().t()).to(bf)
    xn = rmsnorm(h, L.ln2, cfg.rms_eps)
    gu = xn.float() @ L.w_gu.float().t()
    act = (torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]).to(bf)
    return (h.float() + act.float() @ L.w_down.float().t()).to(bf)
