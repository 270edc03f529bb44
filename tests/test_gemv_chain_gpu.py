"""Chained GEMV phases (csrc/kernels/gemv_chain.hip): a decode row's gate_up -> down -> next qkv as
one launch, against the separate launches and the fp32 oracle.

* gate_up and down are bit-identical to ``linear(EPI_SILU)`` + ``linear(EPI_RESADD)``;
* the next layer's q / k / v (RMS norm over 16 waves instead of 12) match ``qkv_rope`` run on the
  chained h within bf16 rounding;
* the hand-off counters re-arm themselves: many launches in a row and HIP-graph replays stay right;
* an engine decoding with the chain (the default for one-row engines) produces the tokens of the
  same engine without it."""

import pytest
import torch

from llm_consensus_amd import ops
from llm_consensus_amd.ops import EPI_RESADD, EPI_SILU, oracle

pytestmark = pytest.mark.gpu

SHAPES = [  # (H, I, nh, nkv, D)
    (1024, 2816, 8, 2, 128),     # llama-small
    (4096, 14336, 32, 8, 128),   # Llama-3-8B
    (3072, 8192, 32, 32, 96),    # Phi-3-mini
]


def _case(H, I, nh, nkv, D, seed, dev="cuda"):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(torch.bfloat16).to(dev)  # noqa: E731
    Nq = (nh + 2 * nkv) * D
    return dict(h=r(1, H), ln2=r(H, sc=0.1) + 1, W_gu=r(2 * I, H, sc=H ** -0.5), W_down=r(H, I, sc=I ** -0.5),
                ln1=r(H, sc=0.1) + 1, W_qkv=r(Nq, H, sc=H ** -0.5))


def _rope_state(nh, nkv, D, bs=64, nb=4, pos=77, dev="cuda"):
    cos_t, sin_t = oracle.rope_tables(torch.tensor([10000.0 ** (-2 * i / D) for i in range(D // 2)]), 1024)
    kc = torch.zeros(nb, nkv, bs, D, dtype=torch.bfloat16, device=dev)
    return dict(cos_t=cos_t.to(dev), sin_t=sin_t.to(dev), kc=kc, vc=torch.zeros_like(kc),
                pos=torch.tensor([pos], dtype=torch.int32, device=dev),
                slots=torch.tensor([2 * bs + pos % bs], dtype=torch.int32, device=dev), q=torch.zeros(1, nh * D,
                                                                                                     dtype=torch.bfloat16,
                                                                                                     device=dev))


@pytest.mark.parametrize("shape", SHAPES)
def test_chain_matches_separate_launches(cuda, shape):
    H, I, nh, nkv, D = shape
    c = _case(H, I, nh, nkv, D, 11)
    ws = ops.gemv_chain_workspace("cuda")
    fault = torch.zeros(1, dtype=torch.int32, device="cuda")
    # reference: separate launches
    h_ref = c["h"].clone()
    act_ref = ops.linear(h_ref, c["W_gu"], EPI_SILU, norm_w=c["ln2"], eps=1e-5)
    ops.linear(act_ref, c["W_down"], EPI_RESADD, out=h_ref)
    rs_ref = _rope_state(nh, nkv, D)
    ops.qkv_rope(h_ref, c["W_qkv"], c["ln1"], 1e-5, rs_ref["q"], rs_ref["kc"], rs_ref["vc"], rs_ref["pos"],
                 rs_ref["slots"], rs_ref["cos_t"], rs_ref["sin_t"], nh, nkv, D, 64)
    for rep in range(3):  # the counters re-arm: every launch of the same workspace is right
        h = c["h"].clone()
        act = torch.zeros(1, I, dtype=torch.bfloat16, device="cuda")
        rs = _rope_state(nh, nkv, D)
        nxt = (c["ln1"], c["W_qkv"], rs["q"], rs["kc"], rs["vc"], rs["pos"], rs["slots"], rs["cos_t"], rs["sin_t"], nh,
               nkv, D, 64)
        ops.gemv_chain(h, c["ln2"], c["W_gu"], act, c["W_down"], 1e-5, ws, fault, nxt if rep != 1 else None)
        torch.cuda.synchronize()
        assert int(fault.item()) == 0
        assert torch.equal(act, act_ref), rep
        assert torch.equal(h, h_ref), rep
        if rep != 1:
            for a, b in ((rs["q"], rs_ref["q"]), (rs["kc"], rs_ref["kc"]), (rs["vc"], rs_ref["vc"])):
                d = (a.float() - b.float()).abs().max().item()
                assert d <= 0.02 * b.float().abs().max().item() + 1e-3, (rep, d)
    # fp32 oracle of the MLP
    hf = c["h"].float()
    xn = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5) * c["ln2"].float()
    gu = xn @ c["W_gu"].float().t()
    a32 = torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]
    h32 = hf + a32 @ c["W_down"].float().t()
    assert (h_ref.float() - h32).abs().max().item() < 0.03 * h32.abs().max().item()


def test_chain_replays_in_a_graph(cuda):
    H, I, nh, nkv, D = SHAPES[0]
    c = _case(H, I, nh, nkv, D, 5)
    ws = ops.gemv_chain_workspace("cuda")
    fault = torch.zeros(1, dtype=torch.int32, device="cuda")
    h = c["h"].clone()
    act = torch.zeros(1, I, dtype=torch.bfloat16, device="cuda")
    rs = _rope_state(nh, nkv, D)
    nxt = (c["ln1"], c["W_qkv"], rs["q"], rs["kc"], rs["vc"], rs["pos"], rs["slots"], rs["cos_t"], rs["sin_t"], nh, nkv,
           D, 64)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ops.gemv_chain(h, c["ln2"], c["W_gu"], act, c["W_down"], 1e-5, ws, fault, nxt)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(4):  # 4 chained launches per replay, each feeding the next
            ops.gemv_chain(h, c["ln2"], c["W_gu"], act, c["W_down"], 1e-5, ws, fault, nxt)
    for rep in range(3):
        h0 = _case(H, I, nh, nkv, D, 100 + rep)["h"]
        h.copy_(h0)
        g.replay()
        torch.cuda.synchronize()
        hr = h0.clone()
        for _ in range(4):
            a = ops.linear(hr, c["W_gu"], EPI_SILU, norm_w=c["ln2"], eps=1e-5)
            ops.linear(a, c["W_down"], EPI_RESADD, out=hr)
        assert torch.equal(h, hr), rep
    assert int(fault.item()) == 0


@pytest.mark.parametrize("name", ["llama-small", "phi3-tiny"])
def test_engine_decode_with_chain_matches_without(cuda, name, monkeypatch):
    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.models.config import FAMILIES

    p = [(i * 13) % 700 + 256 for i in range(60)]
    outs = {}
    for on in ("1", "0"):
        monkeypatch.setenv("LLMC_GEMV_CHAIN", on)
        e = Engine(FAMILIES[name], EngineConfig(device="cuda:0", max_context=1024, seed=7))
        assert e.chain == (on == "1")
        outs[on] = (e.chain, e.generate_ids(p, 48, temperature=0.0, stop_on_eos=False))
        del e
        torch.cuda.empty_cache()
    assert outs["0"][0] is False
    assert outs["1"][1] == outs["0"][1] or _near_tie(name, p, outs)


def _near_tie(name, p, outs):
    """qkv's norm is summed over 16 waves in the chain: a differing greedy token must be a near-tie
    of the unchained engine's own logits."""
    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.models.config import FAMILIES

    a, b = outs["1"][1], outs["0"][1]
    k = next(i for i, (x, y) in enumerate(zip(a, b)) if x != y)
    if k < 8:
        return False
    e = Engine(FAMILIES[name], EngineConfig(device="cuda:0", max_context=1024, seed=7, gemv_chain=False))
    s = e.new_sequence()
    e.prefill([s], [p + b[:k]])
    lt = e.full_logits(s).float().cpu()
    return float(lt.max() - lt[a[k]]) < 0.01 * float(lt.abs().max())
