"""Model-level numerics at full size: teacher-forced per-step decode logits of
the engines the bench and configs 4/5 run, against an fp32 PyTorch forward of the same weights on
the GPU (``ops.oracle.reference_logits``: fp32 math, bf16 only where the engine stores
activations).

* the full 32-layer Llama-3-8B judge at a 13.5k-token context (the bench's judge length at
  4096-token responses; the split-KV attention form with its two-level merge);
* a 2-layer Llama-3-70B tensor-parallel rank's shard (TP=4: 16 query / 2 kv heads, 7168 FFN rows,
  a 32064-row vocab shard) at 2k keys, standing alone as a model;
* a 2-layer, full-width Mixtral-8x7B (8 experts x 14336, top-2) at 2k keys.

The engine side is ``Engine.debug_decode_logits``: greedy tokens and, for token i, the logits it
was sampled from; the oracle runs one causal forward over prompt + tokens[:n - 1] and reads the
logits at every decode position. Tolerance: 2 % of max|logit| against the oracle with the
kernels' bf16 attention probabilities, 3 % against the all-fp32 one (both worst values are
printed; the judge's call `judge.go:96-99` decodes from exactly these logits). At full depth a
random-init 32-layer model amplifies one-ulp bf16 rounding flips of the residual stream, so the
two oracles also differ from each other; that spread (the comparison's own noise floor) is
printed, and past 2 % the bound is 1.25 x the spread. The per-layer test below pins the same
32-layer model with FIXED bounds instead: every layer of one decode step against an fp32 oracle
of that layer alone, fed the engine's own layer input and KV cache, so depth amplification
cannot hide (or excuse) a per-layer defect."""

import pytest
import torch

from llm_consensus_amd.engine import Engine, EngineConfig
from llm_consensus_amd.models.config import FAMILIES
from llm_consensus_amd.ops import oracle

pytestmark = pytest.mark.gpu


def _check(cfg, prompt_len, n=6, seed=5, ctx_extra=64):
    """Worst |engine - oracle| / max|logit| over the n teacher-forced steps, against two oracles:
    the fp32 forward (attention probabilities in f32) and the same forward with the probabilities
    rounded to bf16 before P.V as the MFMA attention kernels round them (row sums f32). The
    second isolates everything else the engine does at full depth; the first is reported too."""
    eng = Engine(cfg, EngineConfig(device="cuda:0", max_context=prompt_len + n + ctx_extra, seed=seed))
    prompt = [(i * 7919) % (cfg.vocab - 512) + 256 for i in range(prompt_len)]
    toks, lg = eng.debug_decode_logits(prompt, n)
    pos = [prompt_len - 1 + i for i in range(n)]
    worst, refs = {}, {}
    for p_bf16 in (False, True):
        ref = oracle.reference_logits(eng.w, cfg, prompt + toks[:n - 1], pos, eng.cos_t, eng.sin_t,
                                      p_bf16=p_bf16).cpu()
        refs[p_bf16] = ref
        w = 0.0
        for i in range(n):
            scale = max(1.0, ref[i].abs().max().item())
            err = (ref[i] - lg[i]).abs().max().item()
            w = max(w, err / scale)
            top2 = torch.topk(ref[i], 2).values
            if (top2[0] - top2[1]).item() > 2 * err:
                assert int(ref[i].argmax()) == toks[i], (cfg.name, i, p_bf16)
        worst["bf16_p" if p_bf16 else "fp32"] = w
    spread = max(((refs[True][i] - refs[False][i]).abs().max() / max(1.0, refs[True][i].abs().max().item())).item()
                 for i in range(n))
    print(f"{cfg.name} ctx {prompt_len}: worst |err| / max|logit| over {n} steps = {worst}; "
          f"oracle spread (fp32 vs bf16-P oracle) {spread:.4f}")
    del eng
    torch.cuda.empty_cache()
    assert worst["bf16_p"] < max(0.02, 1.25 * spread) and worst["fp32"] < max(0.03, 1.25 * spread), (worst, spread)


def test_llama3_8b_full_depth_judge_context(cuda):
    _check(FAMILIES["llama-3-8b"], 13500)


def test_llama3_70b_tp4_rank_shard(cuda):
    b = FAMILIES["llama-3-70b"]
    tp = 4
    cfg = b.with_(name="llama-3-70b-tp4-shard-2l", n_layers=2, n_heads=b.n_heads // tp, n_kv_heads=b.n_kv_heads // tp,
                  intermediate=b.intermediate // tp, vocab=b.vocab // tp)
    _check(cfg, 2048)


def test_mixtral_full_width_two_layers(cuda):
    cfg = FAMILIES["mixtral-8x7b"].with_(name="mixtral-8x7b-2l", n_layers=2)
    _check(cfg, 2048)


def test_llama3_8b_per_layer_at_judge_context(cuda):
    """Each of the 32 layers of one 8B decode step at 13.5k keys against
    ``oracle.reference_decode_layer`` on the engine's own input h and paged K/V: the output error
    is <= 1 % of max|h| and <= 5 % of the layer's own update max|h_out - h_in| (fixed bounds; the
    worst values per layer are printed for profiles/)."""
    cfg = FAMILIES["llama-3-8b"]
    plen = 13500
    eng = Engine(cfg, EngineConfig(device="cuda:0", max_context=plen + 64, seed=5))
    prompt = [(i * 7919) % (cfg.vocab - 512) + 256 for i in range(plen)]
    hs, pos = eng.debug_decode_layers(prompt)
    assert pos == plen and hs.shape == (cfg.n_layers + 1, cfg.hidden)
    rows = []
    for li, L in enumerate(eng.w.layers):
        h_in, out = hs[li:li + 1], hs[li + 1:li + 2].float()
        errs = {}
        for p_bf16 in (True, False):
            ref = oracle.reference_decode_layer(L, cfg, h_in, eng.k_cache[li], eng.v_cache[li], eng.block_tables[0],
                                                pos, eng.cos_t, eng.sin_t, eng.nh, eng.nkv, eng.bs, p_bf16=p_bf16).float()
            d_ref = ref - h_in.float()
            e = (out - ref).abs().max().item()
            errs[p_bf16] = (e / ref.abs().max().item(), e / d_ref.abs().max().item())
        rows.append((li, errs[True][0], errs[True][1], errs[False][0], errs[False][1],
                     hs[li + 1].float().abs().max().item(), (hs[li + 1].float() - hs[li].float()).abs().max().item()))
    print("layer | err/max|h| (bf16-P oracle) | err/max|dh| (bf16-P) | err/max|h| (fp32) | err/max|dh| (fp32) | max|h| | max|dh|")
    for r in rows:
        print(f"{r[0]:2d} | {r[1]:.5f} | {r[2]:.5f} | {r[3]:.5f} | {r[4]:.5f} | {r[5]:.3f} | {r[6]:.3f}")
    worst_h = max(r[1] for r in rows)
    worst_d = max(r[2] for r in rows)
    print(f"worst over {len(rows)} layers: {worst_h:.5f} of max|h|, {worst_d:.5f} of max|dh|")
    del eng
    torch.cuda.empty_cache()
    assert worst_h <= 0.01 and worst_d <= 0.05, (worst_h, worst_d)
