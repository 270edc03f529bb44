"""Microbenchmark of the chained GEMV launch (csrc/kernels/gemv_chain.hip) against separate
launches, Llama-3-8B decode shapes, cold weights (L distinct layers' weights per replay), HIP graphs.

  python scripts/chain_probe.py [--layers 32] [--reps 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_consensus_amd import ops  # noqa: E402
from llm_consensus_amd.ops import EPI_RESADD, EPI_SILU, oracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--layers", type=int, default=32)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--H", type=int, default=4096)
ap.add_argument("--I", type=int, default=14336)
a = ap.parse_args()
H, I, nh, nkv, D, L = a.H, a.I, 32, 8, 128, a.layers
dev = "cuda"
Nq = (nh + 2 * nkv) * D
mk = lambda *s: (torch.randn(*s, device=dev) * 0.02).to(torch.bfloat16)  # noqa: E731
Wgu = [mk(2 * I, H) for _ in range(L)]
Wd = [mk(H, I) for _ in range(L)]
Wq = [mk(Nq, H) for _ in range(L)]
ln = torch.ones(H, dtype=torch.bfloat16, device=dev)
h = mk(1, H)
act = torch.zeros(1, I, dtype=torch.bfloat16, device=dev)
q = torch.zeros(1, nh * D, dtype=torch.bfloat16, device=dev)
kc = torch.zeros(4, nkv, 64, D, dtype=torch.bfloat16, device=dev)
vc = torch.zeros_like(kc)
cos_t, sin_t = oracle.rope_tables([10000.0 ** (-2 * i / D) for i in range(D // 2)], 1024)
cos_t, sin_t = cos_t.to(dev), sin_t.to(dev)
pos = torch.tensor([5], dtype=torch.int32, device=dev)
slots = torch.tensor([69], dtype=torch.int32, device=dev)
ws = ops.gemv_chain_workspace(dev)
fault = torch.zeros(1, dtype=torch.int32, device=dev)


def run(kind):
    for l in range(L):
        if kind == "sep":
            ops.linear(h, Wgu[l], EPI_SILU, out=act, norm_w=ln)
            ops.linear(act, Wd[l], EPI_RESADD, out=h)
            ops.qkv_rope(h, Wq[l], ln, 1e-5, q, kc, vc, pos, slots, cos_t, sin_t, nh, nkv, D, 64)
        elif kind == "sep_mlp":
            ops.linear(h, Wgu[l], EPI_SILU, out=act, norm_w=ln)
            ops.linear(act, Wd[l], EPI_RESADD, out=h)
        elif kind == "gu":
            ops.linear(h, Wgu[l], EPI_SILU, out=act, norm_w=ln)
        elif kind == "down":
            ops.linear(act, Wd[l], EPI_RESADD, out=h)
        elif kind == "qkv":
            ops.qkv_rope(h, Wq[l], ln, 1e-5, q, kc, vc, pos, slots, cos_t, sin_t, nh, nkv, D, 64)
        elif kind.startswith("chain"):
            nxt = (ln, Wq[l], q, kc, vc, pos, slots, cos_t, sin_t, nh, nkv, D, 64) if kind.endswith("qkv") else None
            ops.gemv_chain(h, ln, Wgu[l], act, Wd[l], 1e-5, ws, fault, nxt)


def timeit(kind, unroll=4, flags=0):
    ops.GEMV_CHAIN_DOWN_UNROLL = unroll
    ops.GEMV_CHAIN_FLAGS = flags
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        run(kind)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        run(kind)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / a.reps / L


for kind, u, f in [("gu", 4, 0), ("down", 4, 0), ("qkv", 4, 0), ("sep_mlp", 4, 0), ("sep", 4, 0),
                   ("chain", 4, 0), ("chain", 8, 0), ("chain", 4, 1), ("chain", 4, 0x40),
                   ("chain_qkv", 4, 0), ("chain_qkv", 8, 0), ("chain_qkv", 4, 1), ("chain_qkv", 4, 0x40)]:
    t = timeit(kind, u, f)
    print(f"{kind:10s} unroll {u} flags {f:#x}: {t:7.2f} us per layer", flush=True)
    if f & 1:
        fault.zero_()
        ws.zero_()  # the nowait probe leaves the counters un-re-armed
print("fault", int(fault.item()))
