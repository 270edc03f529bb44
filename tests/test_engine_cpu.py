"""Engine logic on CPU (oracle op path): paged KV across chunked prefills, prefill == incremental
decode logits, batched rows, MoE/Phi-3 families, sampling determinism, cancellation."""

import pytest
import torch

from llm_consensus_amd.context import Context, ContextError
from llm_consensus_amd.engine import Engine, EngineConfig, SamplingParams
from llm_consensus_amd.models.config import FAMILIES
from llm_consensus_amd.models.transformer import TransformerWeights, pair_interleave_heads
from llm_consensus_amd.parallel.comm import TPGroup


def eng(name, **kw):
    kw.setdefault("max_context", 256)
    kw.setdefault("seed", 1)
    return Engine(FAMILIES[name], EngineConfig(device="cpu", **kw))


@pytest.mark.parametrize("name", ["llama-tiny", "mixtral-tiny", "phi3-tiny"])
def test_prefill_equals_incremental(name):
    """Logits after one 40-token prefill == after 25 + 15-token prefills (paged KV reuse)."""
    e = eng(name, block_size=16)
    p = [(i * 31) % 700 + 256 for i in range(40)]
    a = e.new_sequence()
    e.prefill([a], [p])
    la = a.logits.clone()
    e.free_sequence(a)
    b = e.new_sequence()
    e.prefill([b], [p[:25]], want_logits=False)
    e.prefill([b], [p[25:]])
    assert torch.allclose(la, b.logits, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("name", ["llama-tiny", "mixtral-tiny"])
def test_decode_matches_prefill_teacher_forced(name):
    e = eng(name)
    p = [(i * 17) % 700 + 256 for i in range(20)]
    gen = e.generate_ids(p, 6, temperature=0.0, stop_on_eos=False)
    s = e.new_sequence()
    e.prefill([s], [p + gen[:-1]])
    assert int(s.logits.argmax()) == gen[-1]


def test_sampling_determinism_and_seed():
    e = eng("llama-tiny")
    p = list(range(300, 320))
    a = e.generate_ids(p, 10, temperature=1.0, seed=7, stop_on_eos=False)
    b = e.generate_ids(p, 10, temperature=1.0, seed=7, stop_on_eos=False)
    c = e.generate_ids(p, 10, temperature=1.0, seed=8, stop_on_eos=False)
    assert a == b and a != c


def test_batched_rows_match_single():
    e = eng("llama-tiny", max_batch=2)
    p1, p2 = list(range(300, 330)), list(range(500, 512))
    sp = [SamplingParams(8, 0.0, 1.0, 0, 0, False), SamplingParams(8, 0.0, 1.0, 0, 0, False)]
    both = e.generate_batch([p1, p2], sp)
    assert both[0] == e.generate_ids(p1, 8, 0.0, stop_on_eos=False)
    assert both[1] == e.generate_ids(p2, 8, 0.0, stop_on_eos=False)


def test_kv_blocks_freed_and_context_limit():
    e = eng("llama-tiny", max_context=128, block_size=16)
    free0 = e.alloc.num_free
    e.generate_ids(list(range(300, 340)), 10, stop_on_eos=False)
    assert e.alloc.num_free == free0
    with pytest.raises(Exception, match="exceeds engine max_context"):
        e.generate_ids(list(range(300, 420)), 50, stop_on_eos=False)
    assert e.alloc.num_free == free0


def test_cancellation():
    e = eng("llama-tiny")
    ctx = Context.background()
    seen = []

    def cb(ids):
        seen.extend(ids)
        if len(seen) >= 3:
            ctx.cancel()

    with pytest.raises(ContextError, match="context canceled"):
        e.generate_ids(list(range(300, 320)), 50, ctx=ctx, on_tokens=cb, stop_on_eos=False)


def test_pair_interleave_heads():
    rows = torch.arange(2 * 8).view(2 * 8, 1)  # two heads of D=8
    out = pair_interleave_heads(rows, 8).view(-1).tolist()
    assert out == [0, 4, 1, 5, 2, 6, 3, 7, 8, 12, 9, 13, 10, 14, 11, 15]


def test_weights_param_counts():
    c = FAMILIES["llama-3-8b"]
    assert 8.0e9 < c.num_params() < 8.1e9
    assert 70e9 < FAMILIES["llama-3-70b"].num_params() < 71e9
    assert 46e9 < FAMILIES["mixtral-8x7b"].num_params() < 47.5e9
    assert 3.7e9 < FAMILIES["phi-3-mini"].num_params() < 3.9e9
    w = TransformerWeights(FAMILIES["mixtral-tiny"], TPGroup.single(), torch.device("cpu"), 1)
    assert w.layers[0].w_gu.shape == (4, 2 * 384, 256) and w.layers[0].w_router.shape == (4, 256)


def test_attn_buckets_cover_context():
    from llm_consensus_amd.engine.engine import attn_buckets

    for nkv, bph in [(8, 32), (2, 128), (1, 256)]:
        for ctxmax in [100, 1024, 4106, 16394, 131082]:
            bks = attn_buckets(ctxmax, bph, nkv=nkv)
            assert bks[-1][0] == ctxmax
            for cap, chunk, gc, fused in bks:
                if fused:  # fixed 128/256-key chunks cover the bucket; beyond 4k only while <= 256 blocks
                    assert gc * chunk >= cap and chunk in (128, 256)
                    assert cap <= 4096 or gc * nkv <= 256
                else:
                    assert chunk == 128 and cap > 4096 and 1 <= gc <= bph
            assert [b[0] for b in bks] == sorted(b[0] for b in bks)
            split = [b[2] for b in bks if not b[3]]
            assert len(set(split)) == len(split)  # one graph per distinct split grid
    assert attn_buckets(131082, 32)[-1] == (131082, 128, 32, False)
    # Llama-3-8B (8 kv heads): fused up to 8k (256-key chunks at 4k-8k), split above
    assert [(b[1], b[3]) for b in attn_buckets(16394)] == [(128, True), (128, True), (256, True), (256, True),
                                                           (128, False)]
    # a TP=8 rank (one kv head): fused up to 64k keys
    assert all(b[3] for b in attn_buckets(65536, 256, nkv=1))
    assert all(not b[3] for b in attn_buckets(4106, fused_max=0))
    # without GQA (Phi-3: 32 kv heads) buckets above 1k keys use 256-key chunks, split beyond 4k
    assert [(b[1], b[3]) for b in attn_buckets(8200, 16, group=1, nkv=32)] == [(128, True), (256, True), (256, True),
                                                                              (128, False)]


def test_attn_buckets_batching_engine():
    """A batching 8B engine (>= 3 rows, rows x kv heads >= 32) splits a row of L keys into
    min(32, ceil(L / 2048)) ranges whatever its bucket and batch: the grid per head is min(32,
    capacity / 2048), so the kernel's min(grid, ceil(L / 2048)) never depends on the bucket;
    engines of 1-2 rows keep the per-context forms."""
    import math

    from llm_consensus_amd.engine.engine import BATCHING_MIN_KEYS as MK
    from llm_consensus_amd.engine.engine import attn_buckets

    b16 = attn_buckets(131082, 32, rows=16)
    assert all(ch == MK and not fused for _, ch, _, fused in b16)
    assert [(c, g) for c, _, g, _ in b16] == [(2048, 1), (4096, 2), (8192, 4), (16384, 8), (32768, 16),
                                              (131082, 32)]
    assert attn_buckets(131082, 32, rows=4) == b16 == attn_buckets(131082, 32, rows=32)
    # batch invariance: the split a row gets is a function of its own length only
    for L in (1, 700, 2048, 2049, 5000, 13500, 40000, 131000):
        splits = {min(g, math.ceil(L / MK)) for c, _, g, _ in b16 if c >= L}
        assert len(splits) == 1 and splits.pop() == min(32, math.ceil(L / MK)), L
    assert attn_buckets(16394, 32, rows=2) == attn_buckets(16394, 32)
    # fewer than 32 (row, kv head) units (3 duplicate 8B responders: 24; TP ranks with 2 kv
    # heads): still a length-only split, with a 512-key minimum so a row spreads further
    from llm_consensus_amd.engine.engine import BATCHING_MIN_KEYS_FEW as MKF

    for rows, nkv in ((3, 8), (8, 2), (3, 1)):
        bf = attn_buckets(16394, 32, nkv=nkv, rows=rows)
        assert all(ch == MKF and not fused for _, ch, _, fused in bf)
        for L in (1, 511, 513, 2048, 5000, 13500, 16390):
            splits = {min(g, math.ceil(L / MKF)) for c, _, g, _ in bf if c >= L}
            assert len(splits) == 1 and splits.pop() == min(32, math.ceil(L / MKF)), (rows, nkv, L)
    assert attn_buckets(4106, 16, group=1, nkv=32, rows=4) == [(2048, MK, 1, False), (4096, MK, 2, False),
                                                               (4106, MK, 3, False)]  # Phi-3
    assert attn_buckets(200, 32, rows=4) == [(200, MK, 1, False)]


def test_split_blocks_per_head():
    from llm_consensus_amd.engine.engine import split_blocks_per_head

    assert split_blocks_per_head(32, 8) == 32    # Llama-3-8B: 256 blocks per row
    assert split_blocks_per_head(32, 32) == 16   # Phi-3: 512 4-wave blocks
    assert split_blocks_per_head(4, 1) == 256    # a TP=8 rank: every CU, two-level merge
    assert split_blocks_per_head(16, 2) == 128   # a 70B TP=4 rank

def test_engine_rejects_more_rows_than_the_decode_forms_take():
    """32 decode rows per engine (the MFMA form's two token groups), 16 for MoE engines (pairs of
    <= 16 tokens per batched MoE launch): larger engines fail at construction, not mid-decode."""
    import pytest

    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.engine.engine import EngineError
    from llm_consensus_amd.models.config import FAMILIES

    with pytest.raises(EngineError):
        Engine(FAMILIES["mixtral-tiny"], EngineConfig(device="cpu", max_context=64, max_batch=17))
    with pytest.raises(EngineError):
        Engine(FAMILIES["llama-tiny"], EngineConfig(device="cpu", max_context=64, max_batch=33))
    Engine(FAMILIES["llama-tiny"], EngineConfig(device="cpu", max_context=64, max_batch=32))


def test_attn_oproj_bucket_chunks():
    """Keys per block of the fused attention + o_proj launch: the bucket capacity over the grid,
    in 32-key sub-tiles, 0 above 512 keys per block (the kernel's two sub-tiles per wave)."""
    from llm_consensus_amd import ops

    nc = 32
    assert [ops.attn_oproj_chunk(c, nc) for c in (100, 1024, 2048, 4096, 8192, 8193, 16384, 16385)] == \
        [32, 32, 64, 128, 256, 320, 512, 0]
    for cap in range(1, 16385, 97):
        ch = ops.attn_oproj_chunk(cap, nc)
        unit = 64 if ch > 256 else 32  # two sub-tiles per wave above 256 keys: page-aligned 64-key units
        assert ch % unit == 0 and ch * nc >= cap and (ch == 32 or (ch - unit) * nc < cap)
    assert ops.ATTN_OPROJ_MIN_CHUNK <= ops.ATTN_OPROJ_MAX_CHUNK


def test_attn_oproj_cpu_path_is_attention_then_residual_o_proj():
    """The op's CPU path (the oracle) is exactly attention -> o_proj -> += residual on row 0."""
    import math

    from llm_consensus_amd import ops
    from llm_consensus_amd.ops import EPI_RESADD, oracle

    torch.manual_seed(0)
    nh, nkv, D, H, bs, L = 4, 2, 16, 32, 16, 37
    nb = 5
    kc = torch.randn(nb, nkv, bs, D).to(torch.bfloat16)
    vc = torch.randn(nb, nkv, bs, D).to(torch.bfloat16)
    bt = torch.tensor([[3, 0, 4, 1]], dtype=torch.int32)
    sl = torch.tensor([L], dtype=torch.int32)
    q = torch.randn(1, nh * D).to(torch.bfloat16)
    w_o = torch.randn(H, nh * D).to(torch.bfloat16)
    h = torch.randn(1, H).to(torch.bfloat16)
    h1, attn = h.clone(), torch.zeros(1, nh * D, dtype=torch.bfloat16)
    ops.attn_oproj(q, kc, vc, bt, sl, w_o, h1, attn, None, nh, nkv, D, bs, 32, 2, 1 / math.sqrt(D))
    a = oracle.attn_decode(q, kc, vc, bt, sl, nh, nkv, D, bs, 1 / math.sqrt(D))
    h2 = h.clone()
    oracle.linear(a, w_o, EPI_RESADD, h2)
    assert torch.equal(attn, a) and torch.equal(h1, h2)


def test_cpu_engines_never_take_the_fused_attention_oproj():
    eng = Engine(FAMILIES["llama-tiny"], EngineConfig(device="cpu", max_context=256, attn_oproj=True))
    assert eng.ao_nc == 0 and not any(eng.ao_chunks)


def test_debug_decode_layers_matches_per_layer_oracle_cpu():
    """The per-layer decode hook (the full-depth GPU test's instrument) on the CPU path: every
    layer's output equals the one-layer fp32 oracle fed the engine's own input and KV cache to
    within bf16 rounding of the residual stream."""
    from llm_consensus_amd.ops import oracle

    cfg = FAMILIES["llama-tiny"]
    eng = Engine(cfg, EngineConfig(device="cpu", max_context=256, seed=5))
    prompt = [(i * 7919) % (cfg.vocab - 300) + 256 for i in range(100)]
    hs, pos = eng.debug_decode_layers(prompt)
    assert pos == len(prompt) and hs.shape == (cfg.n_layers + 1, cfg.hidden)
    for li, L in enumerate(eng.w.layers):
        ref = oracle.reference_decode_layer(L, cfg, hs[li:li + 1], eng.k_cache[li], eng.v_cache[li], eng.block_tables[0],
                                            pos, eng.cos_t, eng.sin_t, eng.nh, eng.nkv, eng.bs).float()
        err = (hs[li + 1].float() - ref).abs().max().item()
        assert err <= 0.01 * ref.abs().max().item(), (li, err)
