"""The one-launch qkv + attention (csrc/kernels/qkv_attn.hip) on the host: which shapes the kernel
library covers (the engine's per-bucket choice depends on it) and the op's CPU path (qkv_rope +
the attention oracle, what an engine on the CPU would compute)."""

import math

import torch

from llm_consensus_amd import ops
from llm_consensus_amd.ops import oracle


def test_shape_gate():
    from llm_consensus_amd.engine.engine import QKV_ATTN_MAX_ROWS

    # the kernel covers GQA groups 1-8 at D = 64 / 96 / 128 ...
    for nh, nkv, D, K in [(4, 1, 128, 4096),    # Llama-3-8B TP=8
                          (8, 2, 128, 4096),    # Llama-3-8B TP=4
                          (8, 1, 128, 8192),    # Llama-3-70B TP=8
                          (4, 4, 96, 3072),     # Phi-3-mini TP=8
                          (32, 8, 128, 4096)]:  # Llama-3-8B
        assert ops.qkv_attn_supported(nh, nkv, D, K), (nh, nkv, D, K)
    assert not ops.qkv_attn_supported(4, 1, 80, 4096)     # head dim off the MFMA slabs
    assert not ops.qkv_attn_supported(12, 1, 128, 4096)   # G = 12
    # ... and engines take it by default only for the TP ranks' short qkv outputs
    assert (4 + 2) * 128 < QKV_ATTN_MAX_ROWS and (8 + 4) * 128 < QKV_ATTN_MAX_ROWS
    assert (32 + 16) * 128 >= QKV_ATTN_MAX_ROWS


def test_cpu_path_is_qkv_rope_then_attention():
    torch.manual_seed(0)
    nh, nkv, D, K, bs, L = 4, 1, 64, 256, 16, 37
    N = (nh + 2 * nkv) * D
    x = torch.randn(1, K).to(torch.bfloat16)
    nw = torch.ones(K, dtype=torch.bfloat16)
    W = (torch.randn(N, K) / math.sqrt(K)).to(torch.bfloat16)
    nb = 6
    kc = torch.randn(nb, nkv, bs, D).to(torch.bfloat16)
    vc = torch.randn(nb, nkv, bs, D).to(torch.bfloat16)
    bt = torch.tensor([[3, 1, 5, 0, 2]], dtype=torch.int32)
    sl = torch.tensor([L], dtype=torch.int32)
    pos = torch.tensor([L - 1], dtype=torch.int32)
    slots = torch.tensor([int(bt[0, (L - 1) // bs]) * bs + (L - 1) % bs], dtype=torch.int32)
    ang = torch.arange(64, dtype=torch.float32)[:, None] * (1e-2 * torch.arange(D // 2, dtype=torch.float32))[None]
    cos, sin = torch.cos(ang), torch.sin(ang)
    scale = 1 / math.sqrt(D)
    q = torch.zeros(1, nh * D, dtype=torch.bfloat16)
    out = torch.zeros(1, nh * D, dtype=torch.bfloat16)
    kc1, vc1 = kc.clone(), vc.clone()
    ops.qkv_attn(x, W, nw, 1e-5, q, kc1, vc1, pos, slots, cos, sin, bt, sl, out, None, None, None, nh, nkv, D, bs,
                 128, 1, scale)
    q2 = torch.zeros(1, nh * D, dtype=torch.bfloat16)
    kc2, vc2 = kc.clone(), vc.clone()
    ops.qkv_rope(x, W, nw, 1e-5, q2, kc2, vc2, pos, slots, cos, sin, nh, nkv, D, bs)
    ref = oracle.attn_decode(q2, kc2, vc2, bt, sl, nh, nkv, D, bs, scale)
    assert torch.equal(q, q2) and torch.equal(kc1, kc2) and torch.equal(vc1, vc2)
    assert torch.equal(out, ref.to(out.dtype))


def test_engine_plan_policy():
    """Which buckets an engine runs as one qkv + attention launch (engine.qkv_attn_plan)."""
    from llm_consensus_amd.engine.engine import attn_buckets, qkv_attn_plan, split_blocks_per_head

    def plan(nh, nkv, ctx, mode, ao=None):
        b = attn_buckets(ctx, split_blocks_per_head(nh, nkv), 4096, nh // nkv, nkv)
        return b, qkv_attn_plan(b, ao or [0] * len(b), mode, (nh + 2 * nkv) * 128, 64)

    # a TP=8 rank of Llama-3-8B (768 qkv rows): every fused bucket, the bucket's own chunking
    b, (p, _) = plan(4, 1, 20000, "1")
    assert all(q == (ch, gc) for q, (_, ch, gc, fused) in zip(p, b) if fused) and any(p)
    # the whole model (6144 rows) keeps two launches by default ...
    b, (p, _) = plan(32, 8, 9400, "1")
    assert not any(p)
    # ... "all" takes every bucket (the split-form ones as 256-key blocks) and drops attn_oproj there
    ao = [256 if cap >= 4096 else 0 for cap, _, _, _ in b]
    _, (p, ao2) = plan(32, 8, 9400, "all", ao)
    assert all(p) and not any(ao2)
    assert p[-1][0] == 256 and p[-1][1] * 256 >= b[-1][0]
    # default mode never takes a bucket attn_oproj runs
    b, (p, ao2) = plan(4, 1, 9400, "1", [0, 0, 0, 256, 0])
    assert p[3] is None and ao2[3] == 256
    # "0": off
    _, (p, _) = plan(4, 1, 9400, "0")
    assert not any(p)
