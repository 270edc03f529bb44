"""Task timeline of the fused decode layer (csrc/kernels/decode_layer.hip) on one Llama-3-8B layer
at batch 1: per step (qkv / attn / o / gu / down), when its tasks were dispatched, got their task
index, finished waiting for their dependency, computed and signalled (s_memrealtime stamps, 100 MHz),
plus the launch time. Diagnostics for tuning the fused layer; prints a table.

  python scripts/dl_timeline.py --ctx 2048
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_consensus_amd import ops  # noqa: E402
from llm_consensus_amd.engine import Engine, EngineConfig, SamplingParams  # noqa: E402
from llm_consensus_amd.models.config import FAMILIES  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ctx", type=int, default=2048)
ap.add_argument("--model", default="llama-3-8b")
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()

cfg = FAMILIES[a.model].with_(n_layers=2)
e = Engine(cfg, EngineConfig(device="cuda:0", max_context=a.ctx + 64, seed=1, fused_layer=True))
assert e.fused_layer
prompt = [(i * 7919) % 30000 + 256 for i in range(a.ctx)]
s = e.new_sequence()
e.prefill([s], [prompt])
e._reserve(s, s.length + 16)
e._bind_rows([s], [SamplingParams(8, 0.0, 1.0, 0, 0, False)])
e._sample(1, e._gather_logits(1))
torch.cuda.synchronize()
bucket = e._bucket(s.length + 8)
gc = e.layer_gc[bucket]
nh, nkv, D, H, I = e.nh, e.nkv, e.D, cfg.hidden, e.w.inter
def workers(groups):  # as the kernel: about one worker per CU per GEMV step
    return min(groups, 256)


counts = {"qkv": workers((nh + 2 * nkv) * D // 16), "attn": nkv * gc, "o": workers(H // 16),
          "gu": workers(2 * I // 16), "down": workers(H // 16)}
ntask = sum(counts.values())
st = torch.zeros(ntask, 8, dtype=torch.int64, device="cuda")
Lw = e.w.layers[0]


def run(stamps=None):
    ops.decode_layer(Lw, e.h[:1], e.q[:1], e.attn[:1], e.act[:1], e.k_cache[0], e.v_cache[0], e.positions[:1],
                     e.slots[:1], e.seq_lens[:1], e.block_tables[:1], e.cos_t, e.sin_t, e.attn_part, e.attn_counters,
                     e.dl_sync, e.attn_fault, nh, nkv, D, e.bs, gc, cfg.rms_eps, e.scale, stamps=stamps)


for _ in range(5):
    run()
torch.cuda.synchronize()
t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0.record()
for _ in range(a.reps):
    run()
t1.record()
torch.cuda.synchronize()
print(f"{a.model} layer, ctx {a.ctx}, gc {gc}: {1000 * t0.elapsed_time(t1) / a.reps:.1f} us per fused launch "
      f"({ntask} tasks), fault {int(e.attn_fault.item())}")
run(st)
torch.cuda.synchronize()
x = st.cpu().double()
base = x[:, 5].min()
us = (x[:, :6] - base) / 100.0  # 100 MHz ticks -> us
i0 = 0
print(f"{'step':5s} {'tasks':>5s} | {'dispatch':>17s} | {'wait over':>17s} | {'compute':>8s} {'signal':>7s} | "
      f"{'end (max)':>9s} | xcds")
for name, n in counts.items():
    sl = us[i0:i0 + n]
    live = sl[:, 4] > 0  # attention blocks past the context exit without stamps 2-4
    d = sl[:, 5]
    w = sl[live, 2]
    comp = (sl[live, 3] - sl[live, 2]).mean().item() if live.any() else 0.0
    sig = (sl[live, 4] - sl[live, 3]).mean().item() if live.any() else 0.0
    xcd = torch.bincount(x[i0:i0 + n, 7].long(), minlength=8).tolist()
    print(f"{name:5s} {n:5d} | {d.min():7.1f} - {d.max():7.1f} | "
          + (f"{w.min():7.1f} - {w.max():7.1f} | {comp:8.2f} {sig:7.2f} | {sl[live, 4].max():9.1f}" if live.any()
             else " " * 17 + " |")
          + f" | {xcd}")
    i0 += n
print(f"task-index latency (taken - dispatched): mean {(us[:, 0] - us[:, 5]).mean():.2f} us, "
      f"max {(us[:, 0] - us[:, 5]).max():.2f}")
