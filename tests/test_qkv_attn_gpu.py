"""One-launch decode qkv projection + attention (csrc/kernels/qkv_attn.hip) on a real MI355X: against
the two launches it replaces (gemv_qkv_rope + attn_decode fused form: q and the written K/V cache
bit for bit, the attention output within bf16 noise) and the fp32 oracle, over repeated launches on
one workspace (hand-off and merge epochs advance), in a HIP graph replayed at other lengths, and at
the engine level (teacher-forced logits with the launch on and off)."""

import math

import pytest
import torch

from llm_consensus_amd import ops
from llm_consensus_amd.ops import oracle

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def _rope_tables(max_pos, D, theta=500000.0):
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cos(ang).float().cuda(), torch.sin(ang).float().cuda()


class _Case:
    def __init__(self, nh, nkv, D, K, L, bs=64, seed=0):
        torch.manual_seed(seed)
        self.nh, self.nkv, self.D, self.K, self.bs = nh, nkv, D, K, bs
        N = (nh + 2 * nkv) * D
        self.x = torch.randn(1, K, device="cuda").to(BF)
        self.nw = (1 + 0.1 * torch.randn(K, device="cuda")).to(BF)
        self.W = (torch.randn(N, K, device="cuda") / math.sqrt(K)).to(BF)
        nblk = (max(L, 1) + bs - 1) // bs + 2
        nb = nblk + 3
        self.kc = torch.randn(nb, nkv, bs, D, device="cuda").to(BF)
        self.vc = torch.randn(nb, nkv, bs, D, device="cuda").to(BF)
        self.bt = torch.zeros(1, nblk, dtype=torch.int32, device="cuda")
        self.bt[0] = torch.randperm(nb, device="cuda")[:nblk].to(torch.int32)
        self.cos, self.sin = _rope_tables(nblk * bs + 8, D)
        self.sl = torch.zeros(1, dtype=torch.int32, device="cuda")
        self.pos = torch.zeros(1, dtype=torch.int32, device="cuda")
        self.slots = torch.zeros(1, dtype=torch.int32, device="cuda")
        self.set_len(L)

    def set_len(self, L):
        p = L - 1
        self.sl.fill_(L)
        self.pos.fill_(p)
        self.slots.fill_(int(self.bt[0, p // self.bs].item()) * self.bs + p % self.bs)


def _two_launch(cs, kc, vc, chunk, gc, scale):
    nh, nkv, D = cs.nh, cs.nkv, cs.D
    q = torch.zeros(1, nh * D, dtype=BF, device="cuda")
    ops.qkv_rope(cs.x, cs.W, cs.nw, 1e-5, q, kc, vc, cs.pos, cs.slots, cs.cos, cs.sin, nh, nkv, D, cs.bs)
    part, ctr = ops.decode_attn_workspace(1, nh, nkv, D, gc, "cuda", fused=True)
    out = torch.zeros(1, nh * D, dtype=BF, device="cuda")
    ops.attn_decode(q, kc, vc, cs.bt, cs.sl, out, part, ctr, nh, nkv, D, cs.bs, chunk, scale, grid_chunks=gc,
                    fused=True)
    return q, out


def _bucket(L):
    cap = 1024
    while cap < L:
        cap *= 2
    chunk = 128 if cap <= 2048 else 256
    return chunk, cap // chunk


SHAPES = [(4, 1, 128, 4096),   # Llama-3-8B TP=8 rank
          (8, 2, 128, 4096),   # Llama-3-8B TP=4 rank
          (8, 1, 128, 8192),   # Llama-3-70B TP=8 rank
          (4, 4, 96, 3072),    # Phi-3-mini TP=8 rank (no GQA, D = 96)
          (4, 2, 64, 1024),
          (32, 8, 128, 4096),  # Llama-3-8B (LLMC_QKV_ATTN=all)
          (16, 4, 128, 4096)]  # Llama-3-8B TP=2 rank


@pytest.mark.parametrize("nh,nkv,D,K", SHAPES)
@pytest.mark.parametrize("L", [1, 2, 64, 127, 128, 129, 700, 2048, 3001, 7000])
def test_qkv_attn_vs_two_launches_and_oracle(cuda, nh, nkv, D, K, L):
    assert ops.qkv_attn_supported(nh, nkv, D, K)
    cs = _Case(nh, nkv, D, K, L, seed=L + nh)
    chunk, gc = _bucket(L)
    scale = 1 / math.sqrt(D)
    kc_ref, vc_ref = cs.kc.clone(), cs.vc.clone()
    q_ref, out_ref = _two_launch(cs, kc_ref, vc_ref, chunk, gc, scale)
    a_or = oracle.attn_decode(q_ref.cpu(), kc_ref.cpu(), vc_ref.cpu(), cs.bt.cpu(), cs.sl.cpu(), nh, nkv, D, cs.bs,
                              scale).float()
    part, ctr = ops.decode_attn_workspace(1, nh, nkv, D, gc, "cuda", fused=True)
    ws = ops.qkv_attn_workspace(nh, nkv, D, "cuda")
    fault = torch.zeros(1, dtype=torch.int32, device="cuda")
    for _ in range(3):  # one workspace: hand-off and merge epochs advance every launch
        kc, vc = cs.kc.clone(), cs.vc.clone()
        q = torch.zeros(1, nh * D, dtype=BF, device="cuda")
        out = torch.zeros(1, nh * D, dtype=BF, device="cuda")
        ops.qkv_attn(cs.x, cs.W, cs.nw, 1e-5, q, kc, vc, cs.pos, cs.slots, cs.cos, cs.sin, cs.bt, cs.sl, out, part,
                     ctr, ws, nh, nkv, D, cs.bs, chunk, gc, scale, fault=fault)
        torch.cuda.synchronize()
        assert int(fault.item()) == 0
        if (nh + 2 * nkv) * D < 2048:  # the qkv launch's own 4-wave geometry: the same bits
            assert torch.equal(q, q_ref) and torch.equal(kc, kc_ref) and torch.equal(vc, vc_ref)
        else:  # wider outputs: the RMS norm's sum of squares is grouped differently (last bits)
            for a, b in ((q, q_ref), (kc, kc_ref), (vc, vc_ref)):
                assert (a.float() - b.float()).abs().max().item() < 2e-2 * max(1.0, b.float().abs().max().item())
        o = out.float().cpu()
        ref = out_ref.float().cpu()
        tol = 2e-2 * max(1.0, ref.abs().max().item())
        assert (o - ref).abs().max().item() < tol, (o - ref).abs().max().item()
        assert (o - a_or).abs().max().item() < tol
    assert int(ws[1][0].item()) == 0 and int(ws[1][ops.ATTN_CTR_PITCH].item()) == 3  # exits re-armed, 3 epochs


@pytest.mark.parametrize("nh,nkv,D,K", [SHAPES[0], SHAPES[1]])
def test_qkv_attn_graph_replay_at_other_lengths(cuda, nh, nkv, D, K):
    """Captured once for a 2k bucket (128-key chunks x 16), replayed while the length (and so the
    new token's position, slot and the block holding it) changes."""
    Lmax = 2048
    cs = _Case(nh, nkv, D, K, Lmax, seed=3)
    chunk, gc = 128, 16
    scale = 1 / math.sqrt(D)
    part, ctr = ops.decode_attn_workspace(1, nh, nkv, D, gc, "cuda", fused=True)
    ws = ops.qkv_attn_workspace(nh, nkv, D, "cuda")
    fault = torch.zeros(1, dtype=torch.int32, device="cuda")
    kc, vc = cs.kc.clone(), cs.vc.clone()
    q = torch.zeros(1, nh * D, dtype=BF, device="cuda")
    out = torch.zeros(1, nh * D, dtype=BF, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ops.qkv_attn(cs.x, cs.W, cs.nw, 1e-5, q, kc, vc, cs.pos, cs.slots, cs.cos, cs.sin, cs.bt, cs.sl, out, part,
                     ctr, ws, nh, nkv, D, cs.bs, chunk, gc, scale, fault=fault)
    for L in (5, 128, 129, 1500, 2048, 700):
        cs.set_len(L)
        kc.copy_(cs.kc)
        vc.copy_(cs.vc)
        g.replay()
        torch.cuda.synchronize()
        kc_ref, vc_ref = cs.kc.clone(), cs.vc.clone()
        q_ref, out_ref = _two_launch(cs, kc_ref, vc_ref, chunk, gc, scale)
        assert int(fault.item()) == 0
        assert torch.equal(kc, kc_ref) and torch.equal(vc, vc_ref)
        ref = out_ref.float().cpu()
        assert (out.float().cpu() - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item()), L


def test_engine_qkv_attn_matches_two_launch_step(cuda):
    """Engine level (llama-small: 8 q / 2 kv heads x 128, qkv output 1536 rows, covered): teacher-
    forced decode logits with the one-launch qkv + attention against the two launches on the same
    weights, across the 1k and 2k buckets; greedy graph decode == eager."""
    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.models.config import FAMILIES
    from llm_consensus_amd.models.transformer import TransformerWeights
    from llm_consensus_amd.parallel.comm import TPGroup

    cfg = FAMILIES["llama-small"]
    w = TransformerWeights(cfg, TPGroup.single(), torch.device("cuda:0"), seed=31)
    eq = Engine(cfg, EngineConfig(device="cuda:0", max_context=2400, qkv_attn="1"), weights=w)
    e2 = Engine(cfg, EngineConfig(device="cuda:0", max_context=2400, qkv_attn="0"), weights=w)
    assert any(eq.qa_buckets) and not any(e2.qa_buckets)
    for plen in (40, 1030, 2000):
        prompt = [(i * 7919) % (cfg.vocab - 300) + 256 for i in range(plen)]
        ta, la = eq.debug_decode_logits(prompt, 8)
        t2, l2 = e2.debug_decode_logits(prompt, 8)
        for i in range(8):
            if ta[:i] != t2[:i]:  # a near-tie sent the greedy streams apart
                break
            err = (la[i] - l2[i]).abs().max().item()
            assert err < 0.02 * max(1.0, l2[i].abs().max().item()), (plen, i, err)
    prompt = [(i * 31) % 3000 + 256 for i in range(1500)]
    a = eq.generate_ids(prompt, 32, temperature=0.0, stop_on_eos=False)
    ee = Engine(cfg, EngineConfig(device="cuda:0", max_context=2400, qkv_attn="1", use_graphs=False), weights=w)
    b = ee.generate_ids(prompt, 32, temperature=0.0, stop_on_eos=False)
    assert a == b
    assert int(eq.attn_fault.item()) == 0


def test_engine_qkv_attn_all_replaces_attn_oproj(cuda):
    """LLMC_QKV_ATTN=all on a whole Llama-3-8B-shaped model (2 layers): the one launch takes the
    fused buckets, attn_oproj's too; logits match the default engine's."""
    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.models.config import FAMILIES
    from llm_consensus_amd.models.transformer import TransformerWeights
    from llm_consensus_amd.parallel.comm import TPGroup

    cfg = FAMILIES["llama-3-8b"].with_(name="llama-3-8b-2l", n_layers=2)
    w = TransformerWeights(cfg, TPGroup.single(), torch.device("cuda:0"), seed=41)
    ea = Engine(cfg, EngineConfig(device="cuda:0", max_context=8300, qkv_attn="all"), weights=w)
    ed = Engine(cfg, EngineConfig(device="cuda:0", max_context=8300), weights=w)
    assert any(ea.qa_buckets) and not any(ed.qa_buckets)
    assert not any(q and a for q, a in zip(ea.qa_buckets, ea.ao_chunks))
    for plen in (100, 3000, 7000):
        prompt = [(i * 7919) % (cfg.vocab - 300) + 256 for i in range(plen)]
        ta, la = ea.debug_decode_logits(prompt, 6)
        t2, l2 = ed.debug_decode_logits(prompt, 6)
        for i in range(6):
            if ta[:i] != t2[:i]:
                break
            err = (la[i] - l2[i]).abs().max().item()
            assert err < 0.02 * max(1.0, l2[i].abs().max().item()), (plen, i, err)
    assert int(ea.attn_fault.item()) == 0


@pytest.mark.parametrize("nh,nkv,D,K,H", [(4, 1, 128, 4096, 4096),   # 8B TP=8 rank: o_proj K = 512
                                          (8, 2, 128, 4096, 4096),   # 8B TP=4 rank: K = 1024
                                          (16, 4, 128, 4096, 4096),  # 8B TP=2 rank: K = 2048
                                          (16, 16, 96, 3072, 3072),  # Phi-3 TP=2 rank: K = 1536 (3 chunks)
                                          (8, 1, 64, 1024, 1000)])   # a partial last row block
@pytest.mark.parametrize("add_resid", [True, False])
def test_qkv_attn_o_role_matches_the_o_gemv(cuda, nh, nkv, D, K, H, add_resid):
    """The o-role (the token's o_proj in the qkv + attention launch, after every attention block
    has written its head output) against the same launch without it followed by the o GEMV
    (EPI_RESADD / EPI_BF16): the same bits — one row per wave, its 16-B chunks in the same order,
    the same wave sum — launch after launch on one workspace (the o-role's arrival counter and the
    exit count re-arm), at lengths in the one-chunk and the merged forms."""
    scale = 1 / math.sqrt(D)
    torch.manual_seed(5)
    w_o = (torch.randn(H, nh * D, device="cuda") / math.sqrt(nh * D)).to(BF)
    h0 = torch.randn(1, H, device="cuda").to(BF)
    for L in (40, 700, 2000):
        cs = _Case(nh, nkv, D, K, L)
        chunk, gc = _bucket(L)
        part, ctr = ops.decode_attn_workspace(1, nh, nkv, D, gc, "cuda", fused=True)
        ws = ops.qkv_attn_workspace(nh, nkv, D, "cuda")
        fault = torch.zeros(1, dtype=torch.int32, device="cuda")
        for it in range(3):
            kc, vc = cs.kc.clone(), cs.vc.clone()
            q = torch.zeros(1, nh * D, dtype=BF, device="cuda")
            out = torch.zeros(1, nh * D, dtype=BF, device="cuda")
            h = h0.clone()
            ops.qkv_attn(cs.x, cs.W, cs.nw, 1e-5, q, kc, vc, cs.pos, cs.slots, cs.cos, cs.sin, cs.bt, cs.sl, out, part,
                         ctr, ws, nh, nkv, D, cs.bs, chunk, gc, scale, fault=fault, w_o=w_o, h=h, add_resid=add_resid)
            kc2, vc2 = cs.kc.clone(), cs.vc.clone()
            q2 = torch.zeros(1, nh * D, dtype=BF, device="cuda")
            out2 = torch.zeros(1, nh * D, dtype=BF, device="cuda")
            ops.qkv_attn(cs.x, cs.W, cs.nw, 1e-5, q2, kc2, vc2, cs.pos, cs.slots, cs.cos, cs.sin, cs.bt, cs.sl, out2,
                         part, ctr, ws, nh, nkv, D, cs.bs, chunk, gc, scale, fault=fault)
            h2 = h0.clone()
            ops.linear(out2, w_o, ops.EPI_RESADD if add_resid else ops.EPI_BF16, out=h2)
            torch.cuda.synchronize()
            assert int(fault.item()) == 0, (L, it)
            assert torch.equal(out, out2), (L, it)
            assert torch.equal(h, h2), (L, it, (h.float() - h2.float()).abs().max().item())
        c = ws[1].view(-1, ops.ATTN_CTR_PITCH).cpu()
        assert int(c[0, 0]) == 0 and int(c[2, 0]) == 0  # exit count and o-role arrivals re-armed
