"""Decode-step profile harness: one Llama-3-8B engine, prefill + N decode tokens (HIP graphs).
Run under rocprofv3 --kernel-trace --stats to get per-kernel time of the decode step."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from llm_consensus_amd.engine import Engine, EngineConfig
from llm_consensus_amd.models.config import FAMILIES

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama-3-8b")
ap.add_argument("--tokens", type=int, default=128)
ap.add_argument("--prompt", type=int, default=512)
ap.add_argument("--no-graphs", action="store_true")
ap.add_argument("--ctx", type=int, default=8192)
ap.add_argument("--batch", type=int, default=1, help="decode rows per step (continuous-batching engine)")
ap.add_argument("--engine-rows", type=int, default=0, help="engine max_batch (0 = --batch): e.g. one row on a serving engine")
a = ap.parse_args()
cfg = FAMILIES[a.model]
e = Engine(cfg, EngineConfig(device="cuda:0", max_context=a.ctx, seed=1, use_graphs=not a.no_graphs,
                             max_batch=max(a.batch, a.engine_rows)))
prompt = [(i * 7919) % 30000 + 256 for i in range(a.prompt)]
if a.batch > 1:
    from llm_consensus_amd.engine import SamplingParams

    prompts = [[(i * (7919 + 2 * r)) % 30000 + 256 for i in range(a.prompt)] for r in range(a.batch)]
    sp = [SamplingParams(a.tokens, 1.0, 1.0, 0, 100 + r, False) for r in range(a.batch)]
    e.generate_batch(prompts, [SamplingParams(16, 1.0, 1.0, 0, r, False) for r in range(a.batch)])  # warm
    torch.cuda.synchronize()
    t = time.perf_counter()
    outs = e.generate_batch(prompts, sp)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    n = sum(len(o) for o in outs)
    print(f"{a.model}: {a.batch} rows x {a.tokens} tokens in {dt:.3f}s incl prefill of {a.batch} x {a.prompt} -> "
          f"{1000 * dt / a.tokens:.3f} ms/step, {n / dt:.0f} tokens/s", flush=True)
    sys.exit(0)
e.generate_ids(prompt, 16, stop_on_eos=False)  # warm (graph capture)
torch.cuda.synchronize()
t = time.perf_counter()
out = e.generate_ids(prompt, a.tokens, stop_on_eos=False)
torch.cuda.synchronize()
dt = time.perf_counter() - t
print(f"{a.model}: {len(out)} tokens in {dt:.3f}s incl prefill {a.prompt} -> {1000*dt/len(out):.3f} ms/token", flush=True)
# decode-only timing: prefill cost measured separately
s = e.new_sequence(); t = time.perf_counter(); e.prefill([s], [prompt]); torch.cuda.synchronize(); tp = time.perf_counter() - t
e.free_sequence(s)
print(f"prefill {a.prompt} tokens: {1000*tp:.2f} ms -> decode ~{1000*(dt-tp)/len(out):.3f} ms/token", flush=True)
