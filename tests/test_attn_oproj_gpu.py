"""Fused decode attention + o_proj + residual (csrc/kernels/attn_oproj.hip) on a real MI355X:
against the fp32 oracle of the same math, against the two-launch path (attn_decode + o GEMV), over
repeated launches on one workspace (tickets re-armed, epochs advanced), in a HIP graph, and at the
engine level (teacher-forced logits with the fused launch on and off)."""

import math

import pytest
import torch

from llm_consensus_amd import ops
from llm_consensus_amd.engine import Engine, EngineConfig
from llm_consensus_amd.models.config import FAMILIES
from llm_consensus_amd.models.transformer import TransformerWeights
from llm_consensus_amd.ops import EPI_RESADD, oracle
from llm_consensus_amd.parallel.comm import TPGroup

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def _case(L, nh, nkv, D, H, bs=64, seed=0):
    torch.manual_seed(seed)
    nblk = (L + bs - 1) // bs
    nb = nblk + 5
    kc = torch.randn(nb, nkv, bs, D, device="cuda").to(BF)
    vc = torch.randn(nb, nkv, bs, D, device="cuda").to(BF)
    bt = torch.zeros(1, nblk + 4, dtype=torch.int32)
    bt[0, :nblk] = torch.randperm(nb)[:nblk].to(torch.int32)
    q = torch.randn(1, nh * D, device="cuda").to(BF)
    w_o = (torch.randn(H, nh * D, device="cuda") / math.sqrt(nh * D)).to(BF)
    h = torch.randn(1, H, device="cuda").to(BF)
    sl = torch.tensor([L], dtype=torch.int32)
    return kc, vc, bt, sl, q, w_o, h


def _reference(kc, vc, bt, sl, q, w_o, h, nh, nkv, D, bs, scale):
    a = oracle.attn_decode(q.cpu(), kc.cpu(), vc.cpu(), bt, sl, nh, nkv, D, bs, scale)  # bf16 output
    o = a.float() @ w_o.cpu().float().t()
    return a, (h.cpu().float() + o)


@pytest.mark.parametrize("nh,nkv,D,H", [(32, 8, 128, 4096), (8, 2, 128, 1024), (16, 2, 64, 4096)])
@pytest.mark.parametrize("L,cap", [(1, 1024), (31, 1024), (33, 1024), (100, 2048), (1000, 1024), (2048, 2048),
                                   (2100, 4096), (4096, 4096), (5000, 6144), (7999, 8192), (9000, 12288),
                                   (9000, 16384), (13000, 13300),
                                   (16384, 16384)])
def test_attn_oproj_vs_oracle_and_two_launches(cuda, nh, nkv, D, H, L, cap):
    bs = 64
    nc = ops.attn_oproj_grid(H, nh, nkv, D)
    assert nc > 0
    chunk = ops.attn_oproj_chunk(cap, nc)
    if chunk == 0:
        pytest.skip("bucket beyond the fused launch (> 512 keys per block)")
    assert chunk * nc >= L
    kc, vc, bt, sl, q, w_o, h0 = _case(L, nh, nkv, D, H, bs)
    scale = 1 / math.sqrt(D)
    a_ref, h_ref = _reference(kc, vc, bt, sl, q, w_o, h0, nh, nkv, D, bs, scale)
    ws = ops.attn_oproj_workspace(H, nh, nkv, D, nc, "cuda")
    fault = torch.zeros(1, dtype=torch.int32, device="cuda")
    btd, sld = bt.cuda(), sl.cuda()
    # the two-launch path on the same inputs
    part, ctr = ops.decode_attn_workspace(1, nh, nkv, D, 32, "cuda")
    a2 = torch.zeros(1, nh * D, dtype=BF, device="cuda")
    ops.attn_decode(q, kc, vc, btd, sld, a2, part, ctr, nh, nkv, D, bs, 128, scale, grid_chunks=min(32, -(-L // 128)))
    h2 = h0.clone()
    ops.linear(a2, w_o, EPI_RESADD, out=h2)
    for it in range(3):  # one workspace, re-armed by every launch
        h = h0.clone()
        attn = torch.zeros(1, nh * D, dtype=BF, device="cuda")
        ops.attn_oproj(q, kc, vc, btd, sld, w_o, h, attn, ws, nh, nkv, D, bs, chunk, nc, scale, fault=fault)
        torch.cuda.synchronize()
        assert int(fault.item()) == 0
        err_a = (attn.float().cpu() - a_ref.float()).abs().max().item()
        assert err_a < 2e-2, (it, err_a)
        # h: one bf16 rounding of (h + o); o from the same bf16 attention up to its own rounding
        err_h = (h.float().cpu() - h_ref).abs().max().item()
        assert err_h < 2e-2 * max(1.0, h_ref.abs().max().item()), (it, err_h)
        err_2 = (h.float() - h2.float()).abs().max().item()
        assert err_2 < 2e-2 * max(1.0, h_ref.abs().max().item()), (it, err_2)
    # the late-weight variants: each deterministic launch to launch; the merger that defers its
    # weights (3) merges over all 8 waves (four row groups instead of two: another summation
    # order), so 1 and 3 agree to bf16 rounding
    outs = []
    for mode in (1, 3, 1, 3):
        hm = h0.clone()
        am = torch.zeros(1, nh * D, dtype=BF, device="cuda")
        ops.attn_oproj(q, kc, vc, btd, sld, w_o, hm, am, ws, nh, nkv, D, bs, chunk, nc, scale, fault=fault, mode=mode)
        outs.append((hm, am))
    torch.cuda.synchronize()
    assert int(fault.item()) == 0

    def same(a, b):
        return torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])

    def close_runs(a, b):
        tol = 2e-2 * max(1.0, h_ref.abs().max().item())
        return (a[0].float() - b[0].float()).abs().max().item() < tol and \
            (a[1].float() - b[1].float()).abs().max().item() < 2e-2

    assert same(outs[0], outs[2]) and same(outs[1], outs[3]) and close_runs(outs[0], outs[1])
    outs_c = outs
    if nkv == 8 and nh // nkv == 4 and D == 128 and H // nc == 128:
        # whole o_proj rows per block (mode bit 2): no tile partials; with and without the merger
        # deferring its weights the same sums, both against the oracle (own workspace: the tile
        # epoch does not advance in this mode)
        ws2 = ops.attn_oproj_workspace(H, nh, nkv, D, nc, "cuda")
        outs = []
        for mode in (5, 7, 5, 7):
            hm = h0.clone()
            am = torch.zeros(1, nh * D, dtype=BF, device="cuda")
            ops.attn_oproj(q, kc, vc, btd, sld, w_o, hm, am, ws2, nh, nkv, D, bs, chunk, nc, scale, fault=fault,
                           mode=mode)
            outs.append((hm, am))
        torch.cuda.synchronize()
        assert int(fault.item()) == 0
        assert same(outs[0], outs[2]) and same(outs[1], outs[3]) and close_runs(outs[0], outs[1])
        assert torch.equal(outs[0][1], outs_c[0][1])  # the attention itself is the same launch's
        assert torch.equal(outs[1][1], outs_c[1][1])
        err_fr = (outs[0][0].float().cpu() - h_ref).abs().max().item()
        assert err_fr < 2e-2 * max(1.0, h_ref.abs().max().item()), err_fr
    _, _, tile_part, counters = ws
    c = counters.view(-1, 16).cpu()
    # head tickets and tile tickets re-armed, the exit counter re-armed; the head epoch advanced by
    # all 7 launches, the tile epoch by those with tile partials (not the default's whole rows)
    whole_rows = bool(ops.ATTN_OPROJ_MODE & 4) and nkv == 8 and nh // nkv == 4 and D == 128 and H // nc == 128
    assert int(c[: nkv + nc, 0].abs().sum()) == 0 and int(c[nkv + nc, 0]) == 0, c[:, :2]
    assert int(c[:nkv, 2:4].abs().sum()) == 0, c[:nkv, :4]  # the u64 head tickets re-armed
    assert torch.equal(c[:nkv, 1], torch.full((nkv,), 7, dtype=torch.int32))
    assert int(c[nkv + nc, 1]) == (4 if whole_rows else 7)


def test_attn_oproj_shape_gates(cuda):
    """Shapes the kernel rejects are never handed to it: more kv heads than one o_proj row sums
    (kAoMaxKv = 8) give no grid, and an engine with 32-key pages keeps the two launches in every
    bucket that would need > 256 keys per block (two 32-key sub-tiles of one 64-key unit per wave)."""
    assert ops.attn_oproj_grid(4096, 64, 8, 64) > 0
    assert ops.attn_oproj_grid(4096, 128, 16, 64) == 0  # G * D = 512 but 16 kv heads
    cfg = FAMILIES["llama-small"]
    e = Engine(cfg, EngineConfig(device="cuda:0", max_context=16384, block_size=32, attn_oproj=True,
                                 attn_oproj_min_chunk=32))
    if e.ao_nc:
        chunks = [ops.attn_oproj_chunk(cap, e.ao_nc) for cap, _, _, _ in e.attn_buckets]
        assert any(ch > 256 for ch in chunks)
        for ch, used in zip(chunks, e.ao_chunks):
            assert used == (ch if 0 < ch <= 256 else 0), (chunks, e.ao_chunks)


def test_attn_oproj_graph_replay_and_length_changes(cuda):
    """Captured once, replayed while the length grows across chunk boundaries (blocks without keys
    still take their tickets and do their o_proj rows)."""
    nh, nkv, D, H, bs = 32, 8, 128, 4096, 64
    nc = ops.attn_oproj_grid(H, nh, nkv, D)
    cap = 2048
    chunk = ops.attn_oproj_chunk(cap, nc)
    kc, vc, bt, sl, q, w_o, h0 = _case(cap, nh, nkv, D, H, bs, seed=5)
    scale = 1 / math.sqrt(D)
    ws = ops.attn_oproj_workspace(H, nh, nkv, D, nc, "cuda")
    fault = torch.zeros(1, dtype=torch.int32, device="cuda")
    btd = bt.cuda()
    sld = torch.tensor([1], dtype=torch.int32, device="cuda")
    h = h0.clone()
    attn = torch.zeros(1, nh * D, dtype=BF, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.attn_oproj(q, kc, vc, btd, sld, w_o, h, attn, ws, nh, nkv, D, bs, chunk, nc, scale, fault=fault)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.attn_oproj(q, kc, vc, btd, sld, w_o, h, attn, ws, nh, nkv, D, bs, chunk, nc, scale, fault=fault)
    for L in (5, 64, 65, 700, 1023, 2048):
        sld.fill_(L)
        h.copy_(h0)
        g.replay()
        torch.cuda.synchronize()
        _, h_ref = _reference(kc, vc, bt, torch.tensor([L], dtype=torch.int32), q, w_o, h0, nh, nkv, D, bs, scale)
        err = (h.float().cpu() - h_ref).abs().max().item()
        assert err < 2e-2 * max(1.0, h_ref.abs().max().item()), (L, err)
    assert int(fault.item()) == 0


@pytest.mark.parametrize("name,plen", [("llama-small", 90), ("llama-small", 1500), ("llama-small", 5000)])
def test_engine_attn_oproj_matches_two_launch_step(cuda, name, plen, monkeypatch):
    """Teacher-forced decode logits of a one-row engine with the fused attention + o_proj launch
    (in every bucket it covers: LLMC_ATTN_OPROJ=all) against the same weights on the two-launch
    step; graph replay == eager for the fused path."""
    monkeypatch.setenv("LLMC_ATTN_OPROJ", "all")
    cfg = FAMILIES[name]
    w = TransformerWeights(cfg, TPGroup.single(), torch.device("cuda:0"), seed=21)
    ctx = plen + 64
    ea = Engine(cfg, EngineConfig(device="cuda:0", max_context=ctx, attn_oproj=True), weights=w)
    e2 = Engine(cfg, EngineConfig(device="cuda:0", max_context=ctx, attn_oproj=False), weights=w)
    assert ea.ao_nc > 0 and any(ea.ao_chunks) and e2.ao_nc == 0
    prompt = [(i * 7919) % (cfg.vocab - 300) + 256 for i in range(plen)]
    n = 10
    ta, la = ea.debug_decode_logits(prompt, n)
    t2, l2 = e2.debug_decode_logits(prompt, n)
    for i in range(n):
        if ta[:i] != t2[:i]:  # a near-tie sent the greedy streams apart
            break
        err = (la[i] - l2[i]).abs().max().item()
        assert err < 0.02 * max(1.0, l2[i].abs().max().item()), (i, err)
    a = ea.generate_ids(prompt, 24, temperature=0.8, seed=7, stop_on_eos=False)
    ee = Engine(cfg, EngineConfig(device="cuda:0", max_context=ctx, attn_oproj=True, use_graphs=False), weights=w)
    b = ee.generate_ids(prompt, 24, temperature=0.8, seed=7, stop_on_eos=False)
    assert a == b
    assert int(ea.attn_fault.item()) == 0


@pytest.mark.parametrize("nh,nkv,D,H", [(4, 1, 128, 4096), (8, 2, 128, 4096), (16, 4, 128, 4096)])
@pytest.mark.parametrize("L,cap", [(7, 1024), (1000, 1024), (2048, 2048), (3000, 4096)])
@pytest.mark.parametrize("add_resid", [True, False])
def test_attn_oproj_tp_rank_shapes(cuda, nh, nkv, D, H, L, cap, add_resid):
    """The Llama-3-8B TP=8 / 4 / 2 rank shapes (1-4 kv heads, the tile-reduce form) vs the fp32
    oracle: rank 0 adds its share to the residual, the other ranks' launches write the share alone
    (their all-reduce follows; the fused all-reduce epilogue is covered by tests/test_tp_gpu.py)."""
    bs = 64
    nc = ops.attn_oproj_grid(H, nh, nkv, D)
    assert nc > 0
    chunk = ops.attn_oproj_chunk(cap, nc)
    assert chunk and chunk * nc >= L
    kc, vc, bt, sl, q, w_o, h0 = _case(L, nh, nkv, D, H, bs)
    scale = 1 / math.sqrt(D)
    a_ref, h_ref = _reference(kc, vc, bt, sl, q, w_o, h0, nh, nkv, D, bs, scale)
    if not add_resid:
        h_ref = h_ref - h0.cpu().float()
    ws = ops.attn_oproj_workspace(H, nh, nkv, D, nc, "cuda")
    fault = torch.zeros(1, dtype=torch.int32, device="cuda")
    for it in range(2):
        h = h0.clone()
        attn = torch.zeros(1, nh * D, dtype=BF, device="cuda")
        ops.attn_oproj(q, kc, vc, bt.cuda(), sl.cuda(), w_o, h, attn, ws, nh, nkv, D, bs, chunk, nc, scale, fault=fault,
                       add_resid=add_resid)
        torch.cuda.synchronize()
        assert int(fault.item()) == 0
        assert (attn.float().cpu() - a_ref.float()).abs().max().item() < 2e-2
        err_h = (h.float().cpu() - h_ref).abs().max().item()
        assert err_h < 2e-2 * max(1.0, h_ref.abs().max().item()), (it, err_h)


@pytest.mark.parametrize("nh,nkv,D,H", [(32, 8, 128, 4096), (8, 2, 128, 1024)])
@pytest.mark.parametrize("L,cap", [(100, 2048), (2048, 2048), (9000, 16384)])
def test_attn_oproj_weight_gate_is_timing_only(cuda, nh, nkv, D, H, L, cap):
    """Mode bit 3 (the grid-wide weight gate: no block requests its o_proj weights before every
    block has streamed its K/V) changes when loads issue, never what is computed: the same bits as
    the ungated mode, launch after launch on one workspace (the gate's epoch re-arms itself)."""
    bs = 64
    nc = ops.attn_oproj_grid(H, nh, nkv, D)
    chunk = ops.attn_oproj_chunk(cap, nc)
    if chunk == 0:
        pytest.skip("bucket beyond the fused launch")
    kc, vc, bt, sl, q, w_o, h0 = _case(L, nh, nkv, D, H, bs)
    scale = 1 / math.sqrt(D)
    fault = torch.zeros(1, dtype=torch.int32, device="cuda")
    fr = nkv == 8 and nh // nkv == 4 and D == 128 and H // nc == 128
    base = 7 if fr else 3
    ws = ops.attn_oproj_workspace(H, nh, nkv, D, nc, "cuda")
    outs = []
    for mode in (base, base | 8, base | 8, base, base | 8):
        hm = h0.clone()
        am = torch.zeros(1, nh * D, dtype=BF, device="cuda")
        ops.attn_oproj(q, kc, vc, bt.cuda(), sl.cuda(), w_o, hm, am, ws, nh, nkv, D, bs, chunk, nc, scale, fault=fault,
                       mode=mode)
        outs.append((hm, am))
    torch.cuda.synchronize()
    assert int(fault.item()) == 0
    for o in outs[1:]:
        assert torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1])
    c = ws[3].view(-1, 16).cpu()
    assert int(c[nkv + nc + 1, 0]) == 0 and int(c[nkv + nc + 1, 1]) == 3  # arrivals re-armed, 3 gated launches


@pytest.mark.parametrize("L,cap", [(100, 2048), (2048, 2048), (5000, 8192), (9000, 16384)])
def test_attn_oproj_fused_moe_router(cuda, L, cap):
    """Mixtral's attention shape (32 q / 8 kv heads x 128, H 4096; 8 experts, top 2): the decode
    router inside the whole-row attention + o_proj launch. h and the attention output are the bits
    of the launch without it; the ids are moe_router's on that h (and the fp32 oracle's top 2), the
    weights agree to f32 rounding (another summation order), the expert gate_up GEMV on them is the
    bits of the one on moe_router's ids; launch after launch (the epoch advances) and from a HIP
    graph the same bits."""
    nh, nkv, D, H, bs, E, k, eps, inter = 32, 8, 128, 4096, 64, 8, 2, 1e-5, 1024
    nc = ops.attn_oproj_grid(H, nh, nkv, D)
    chunk = ops.attn_oproj_chunk(cap, nc)
    assert chunk and ops.attn_oproj_form(H, nh, nkv, D, nc, chunk) == 2
    assert ops.attn_oproj_form(H, nh, nkv, D, nc, chunk, mode=3) == 1  # tile form: no partials there
    kc, vc, bt, sl, q, w_o, h0 = _case(L, nh, nkv, D, H, bs, seed=3)
    scale = 1 / math.sqrt(D)
    g = torch.Generator(device="cuda").manual_seed(11)
    norm_w = (1 + 0.1 * torch.randn(H, device="cuda", generator=g)).to(BF)
    W_r = (torch.randn(E, H, device="cuda", generator=g) / math.sqrt(H)).to(BF)
    W_gu = (torch.randn(E, 2 * inter, H, device="cuda", generator=g) / math.sqrt(H)).to(BF)
    ws = ops.attn_oproj_workspace(H, nh, nkv, D, nc, "cuda")
    rws = ops.attn_oproj_router_workspace(nkv, nc, "cuda")
    fault = torch.zeros(1, dtype=torch.int32, device="cuda")
    btd, sld = bt.cuda(), sl.cuda()
    h_ref = h0.clone()
    a_ref = torch.zeros(1, nh * D, dtype=BF, device="cuda")
    ops.attn_oproj(q, kc, vc, btd, sld, w_o, h_ref, a_ref, ws, nh, nkv, D, bs, chunk, nc, scale, fault=fault)
    w_ref = torch.zeros(1, k, dtype=torch.float32, device="cuda")
    ids_ref = torch.zeros(1, k, dtype=torch.int32, device="cuda")
    ops.moe_router(h_ref, norm_w, eps, W_r, k, w_ref, ids_ref)
    act_ref = torch.zeros(k, inter, dtype=BF, device="cuda")
    ops.moe_gemv(h_ref, W_gu, ids_ref, k, act_ref, 2 * inter, H, ops.EPI_SILU, norm_w=norm_w, eps=eps)
    torch.cuda.synchronize()
    # fp32 oracle of the logits on that h: its top 2 (skip the id checks on a near-tie)
    hf = h_ref.float().cpu()
    xn = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps) * norm_w.float().cpu()
    lg = (xn @ W_r.float().cpu().t())[0]
    top = torch.sort(lg, descending=True)
    tie = float(top.values[k - 1] - top.values[k]) < 1e-3

    h = h0.clone()
    a = torch.zeros(1, nh * D, dtype=BF, device="cuda")
    w = torch.zeros(1, k, dtype=torch.float32, device="cuda")
    ids = torch.zeros(1, k, dtype=torch.int32, device="cuda")
    act = torch.zeros(k, inter, dtype=BF, device="cuda")

    def launch():
        ops.attn_oproj(q, kc, vc, btd, sld, w_o, h, a, ws, nh, nkv, D, bs, chunk, nc, scale, fault=fault,
                       router=(norm_w, W_r, eps, k, w, ids, rws))
        ops.moe_gemv(h, W_gu, ids, k, act, 2 * inter, H, ops.EPI_SILU, norm_w=norm_w, eps=eps)

    def check(tag):
        assert int(fault.item()) == 0
        assert torch.equal(h, h_ref) and torch.equal(a, a_ref), tag
        if not tie:
            assert torch.equal(ids, ids_ref), (tag, ids, ids_ref)
            assert sorted(ids[0].tolist()) == sorted(top.indices[:k].tolist())
            assert torch.equal(act, act_ref), tag
        assert (w - w_ref).abs().max().item() < 1e-3, (tag, w, w_ref)
        assert abs(float(w.sum()) - 1.0) < 1e-5

    outs = []
    for it in range(3):
        h.copy_(h0)
        w.fill_(-1.0)
        ids.fill_(-1)
        act.zero_()
        launch()
        torch.cuda.synchronize()
        check(it)
        assert int(rws[1][0].item()) == it + 1  # the epoch advanced once per launch
        outs.append((ids.clone(), w.clone(), act.clone()))
    for o in outs[1:]:
        assert all(torch.equal(x, y) for x, y in zip(o, outs[0]))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        launch()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        launch()
    for it in range(3):
        h.copy_(h0)
        w.zero_()
        ids.zero_()
        act.zero_()
        gr.replay()
        torch.cuda.synchronize()
        check(("graph", it))
        assert torch.equal(ids, outs[0][0]) and torch.equal(w, outs[0][1]) and torch.equal(act, outs[0][2])


def test_engine_fused_moe_router_matches_router_launch(cuda):
    """A two-layer Mixtral-8x7B-shaped engine (the whole-row attention + o_proj form needs its H =
    4096): teacher-forced greedy logits with the router folded into the attention + o_proj launch
    against the router's own launch, same weights; graph replay == eager with the fold."""
    cfg = FAMILIES["mixtral-8x7b"].with_(name="mixtral-8x7b-2l", n_layers=2)
    w = TransformerWeights(cfg, TPGroup.single(), torch.device("cuda:0"), seed=5)
    plen = 300
    ctx = plen + 64
    ea = Engine(cfg, EngineConfig(device="cuda:0", max_context=ctx, attn_oproj=True, attn_oproj_min_chunk=32,
                                  ao_router=True), weights=w)
    eb = Engine(cfg, EngineConfig(device="cuda:0", max_context=ctx, attn_oproj=True, attn_oproj_min_chunk=32,
                                  ao_router=False), weights=w)
    assert any(ea.ao_router) and not any(eb.ao_router)
    prompt = [(i * 7919) % (cfg.vocab - 300) + 256 for i in range(plen)]
    n = 8
    ta, la = ea.debug_decode_logits(prompt, n)
    tb, lb = eb.debug_decode_logits(prompt, n)
    for i in range(n):
        if ta[:i] != tb[:i]:  # a near-tie sent the greedy streams apart
            break
        err = (la[i] - lb[i]).abs().max().item()
        assert err < 0.02 * max(1.0, lb[i].abs().max().item()), (i, err)
    a = ea.generate_ids(prompt, 16, temperature=0.8, seed=7, stop_on_eos=False)
    ee = Engine(cfg, EngineConfig(device="cuda:0", max_context=ctx, attn_oproj=True, attn_oproj_min_chunk=32,
                                  ao_router=True, use_graphs=False), weights=w)
    b = ee.generate_ids(prompt, 16, temperature=0.8, seed=7, stop_on_eos=False)
    assert a == b
    assert int(ea.attn_fault.item()) == 0


@pytest.mark.parametrize("nh,nkv,D,H", [(32, 8, 128, 4096), (8, 2, 128, 1024)])
@pytest.mark.parametrize("L,cap", [(100, 2048), (2048, 2048), (9000, 16384)])
def test_attn_oproj_l2_copy_is_timing_only(cuda, nh, nkv, D, H, L, cap):
    """The same-XCD L2 copy of the attention partials (default) vs mode bit 5 (the merger always
    reads the write-through copy): the same bits, launch after launch on one workspace."""
    bs = 64
    nc = ops.attn_oproj_grid(H, nh, nkv, D)
    chunk = ops.attn_oproj_chunk(cap, nc)
    if chunk == 0:
        pytest.skip("bucket beyond the fused launch")
    kc, vc, bt, sl, q, w_o, h0 = _case(L, nh, nkv, D, H, bs)
    scale = 1 / math.sqrt(D)
    fault = torch.zeros(1, dtype=torch.int32, device="cuda")
    fr = nkv == 8 and nh // nkv == 4 and D == 128 and H // nc == 128
    base = 7 if fr else 3
    ws = ops.attn_oproj_workspace(H, nh, nkv, D, nc, "cuda")
    outs = []
    for mode in (base, base | 32, base, base | 32, base):
        hm = h0.clone()
        am = torch.zeros(1, nh * D, dtype=BF, device="cuda")
        ops.attn_oproj(q, kc, vc, bt.cuda(), sl.cuda(), w_o, hm, am, ws, nh, nkv, D, bs, chunk, nc, scale, fault=fault,
                       mode=mode)
        outs.append((hm, am))
    torch.cuda.synchronize()
    assert int(fault.item()) == 0
    for o in outs[1:]:
        assert torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1])
