"""Decode time of ONE tensor-parallel rank's shard of Llama-3-8B (all 32 layers), alone on one GPU:
the compute floor of the TP judge's decode step at TP=2/4/8 (heads, KV heads, FFN rows and vocab
divided by tp), without the all-reduces. Used to project the judge phase of bench.py's N-GPU run
(which this environment cannot launch) and to see how much of a shard's step is per-kernel
overhead rather than weight streaming.

  python scripts/tp_shard_decode.py --tp 1,2,4,8 --ctx 2048,33000 --tokens 256
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_consensus_amd.engine import Engine, EngineConfig  # noqa: E402
from llm_consensus_amd.models.config import FAMILIES  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tp", default="1,2,4,8")
ap.add_argument("--ctx", default="2048,33000")
ap.add_argument("--tokens", type=int, default=256)
ap.add_argument("--model", default="llama-3-8b")
a = ap.parse_args()

base = FAMILIES[a.model]
for tp in [int(t) for t in a.tp.split(",")]:
    cfg = base.with_(name=f"{a.model}-tp{tp}-shard", n_heads=base.n_heads // tp, n_kv_heads=base.n_kv_heads // tp,
                     intermediate=base.intermediate // tp, vocab=base.vocab // tp)
    ctxs = [int(c) for c in a.ctx.split(",")]
    e = Engine(cfg, EngineConfig(device="cuda:0", max_context=max(ctxs) + a.tokens + 64, seed=1))
    e.warmup_graphs()
    mb = cfg.active_weight_bytes() / 1e6
    for ctx in ctxs:
        prompt = [(i * 7919) % (cfg.vocab - 512) + 256 for i in range(ctx)]
        s = e.new_sequence()
        e.prefill([s], [prompt])
        torch.cuda.synchronize()
        e.free_sequence(s)
        e.generate_ids(prompt[:64], 16, stop_on_eos=False)  # warm
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = e.generate_ids(prompt, a.tokens, stop_on_eos=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        s = e.new_sequence()
        t = time.perf_counter()
        e.prefill([s], [prompt])
        torch.cuda.synchronize()
        tp_s = time.perf_counter() - t
        e.free_sequence(s)
        ms = 1000 * (dt - tp_s) / len(out)
        print(f"{a.model} tp={tp} ctx={ctx}: decode {ms:.3f} ms/token ({mb:.0f} MB streamed/token -> "
              f"{mb / 1e3 / ms:.2f} TB/s effective), prefill {ctx} tokens {1000 * tp_s:.1f} ms", flush=True)
    del e
    torch.cuda.empty_cache()
