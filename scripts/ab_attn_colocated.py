"""A/B of the decode-attention form for CO-LOCATED responder engines (bench.py round, one GPU).

Hypothesis: when three engines share the GPU, attention latency is hidden by the other engines'
weight streaming, so what counts is the CU time a form occupies; fewer split blocks per kv head
(less prologue/merge work) might raise the round's aggregate throughput even though each launch
is slower alone. Usage: python scripts/ab_attn_colocated.py VARIANT [bench.py args]
VARIANT: base | g8 | g4 | c256 (responder engines only: max_context < 16k; the judge keeps the default).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import llm_consensus_amd.engine.engine as em  # noqa: E402

variant = sys.argv.pop(1)
_orig = em.attn_buckets


def patched(ctxmax, blocks_per_head=32, fused_max=4096, group=4, nkv=8, rows=1):
    if ctxmax >= 16384 or variant == "base":
        return _orig(ctxmax, blocks_per_head, fused_max, group, nkv, rows)
    if variant in ("g8", "g4"):
        return _orig(ctxmax, int(variant[1:]), 0, group, nkv, rows)
    if variant == "c256":
        out, cap = [], 1024
        while True:
            c = min(cap, ctxmax)
            out.append((c, 256, (c + 255) // 256, True))
            if cap >= ctxmax:
                return out
            cap *= 2
    raise SystemExit(f"unknown variant {variant}")


em.attn_buckets = patched
sys.argv[0] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
import runpy  # noqa: E402

runpy.run_path(sys.argv[0], run_name="__main__")
