"""Probe of the decode-attention fault word (a merger that gave up on a partial) under the
microbenchmark's pattern: many K/V copies cycled through one workspace, eager warmup, graph
capture, replays. Prints the fault word after each stage and the time per call.

  python scripts/attn_fault_probe.py
"""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_consensus_amd import ops  # noqa: E402

BF = torch.bfloat16


def case(L, nh, nkv, D, bs=64):
    nb = (L + bs - 1) // bs + 2
    kc = torch.randn(nb, nkv, bs, D, device="cuda").to(BF)
    vc = torch.randn_like(kc)
    per = (L + bs - 1) // bs
    bt = torch.randperm(nb, device="cuda")[:per].view(1, per).to(torch.int32)
    sl = torch.full((1,), L, dtype=torch.int32, device="cuda")
    q = torch.randn(1, nh * D, device="cuda").to(BF)
    out = torch.empty(1, nh * D, dtype=BF, device="cuda")
    return kc, vc, bt, sl, q, out


def probe(L, chunk, gc, max_chunks, copies=13, nh=32, nkv=8, D=128):
    cases = [case(L, nh, nkv, D) for _ in range(copies)]
    part, ctr = ops.decode_attn_workspace(1, nh, nkv, D, max_chunks, "cuda")
    fault = torch.zeros(1, dtype=torch.int32, device="cuda")
    sc = 1 / math.sqrt(D)
    it = [0]

    def fn():
        kc, vc, bt, sl, q, out = cases[it[0] % copies]
        ops.attn_decode(q, kc, vc, bt, sl, out, part, ctr, nh, nkv, D, 64, chunk, sc, grid_chunks=gc, fused=True,
                        fault=fault)
        it[0] += 1

    report = []
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    report.append(("eager", int(fault.item())))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(5):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    report.append(("side-stream", int(fault.item())))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(39):
            fn()
    torch.cuda.synchronize()
    report.append(("captured", int(fault.item())))
    t0 = time.perf_counter()
    for r in range(10):
        g.replay()
        torch.cuda.synchronize()
        report.append((f"replay{r}", int(fault.item())))
    dt = (time.perf_counter() - t0) / 390 * 1e6
    ref = None
    print(f"L={L} chunk={chunk} gc={gc} max_chunks={max_chunks}: {dt:.1f} us/call (host-timed) faults "
          + " ".join(f"{k}={v}" for k, v in report) + f" ctr={ctr[0, :, :2].flatten().tolist()[:6]}", flush=True)


if __name__ == "__main__":
    for L, chunk, gc in [(4096, 256, 16), (4095, 256, 16), (4000, 256, 16), (2048, 128, 16), (4096, 128, 32)]:
        for mc in (gc, 32):
            probe(L, chunk, gc, mc)
