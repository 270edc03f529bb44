"""Micro-benchmarks of individual decode kernels (device time via HIP events over many launches).

Usage: python scripts/microbench_kernels.py [attn|gemv|all]
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from llm_consensus_amd import ops

BF = torch.bfloat16


def timeit(fn, iters=50, warm=5):
    """Device time per call: `iters` calls captured in one HIP graph, replayed 10x (no host
    launch overhead; includes the inter-kernel boundary as in the real decode graph)."""
    s = torch.cuda.Stream()
    # the side stream must see every buffer the default stream initialised (a workspace still being
    # zeroed when the first launches ran left stale counters: a merger then gave up on a partial)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warm):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / (10 * iters)  # us


def _attn_case(L, nh, nkv, D, bs=64, B=1):
    nb = B * ((L + bs - 1) // bs) + 2
    kc = torch.randn(nb, nkv, bs, D, device="cuda").to(BF)
    vc = torch.randn_like(kc)
    per = (L + bs - 1) // bs
    bt = torch.randperm(nb, device="cuda")[: B * per].view(B, per).to(torch.int32)
    sl = torch.full((B,), L, dtype=torch.int32, device="cuda")
    q = torch.randn(B, nh * D, device="cuda").to(BF)
    out = torch.empty(B, nh * D, dtype=BF, device="cuda")
    return kc, vc, bt, sl, q, out


def bench_attn(shapes=((32, 8, 128), (32, 32, 96), (16, 2, 128), (8, 1, 128), (4, 1, 128))):
    """Decode attention per layer (graph-timed, random paged K/V): the fused form (fixed 128/256-key
    chunk blocks over the power-of-two bucket capacity) vs the balanced split over its grid sizes
    (blocks per kv head); both merge in-launch."""
    for nh, nkv, D in shapes:
        for L in [128, 600, 1024, 2048, 4096, 8192, 16384, 33000]:
            kc, vc, bt, sl, q, out = _attn_case(L, nh, nkv, D)
            sc = 1 / math.sqrt(D)
            gb = L * nkv * D * 2 * 2 / 1e9
            line = []
            best = 1e9
            cap = 1024
            while cap < L:
                cap *= 2
            for ch in (128, 256):
                if (cap // ch) * nkv > 1024:  # beyond two residency rounds: not a candidate
                    continue
                gc = cap // ch
                part, ctr = ops.decode_attn_workspace(1, nh, nkv, D, gc, "cuda", fused=True)
                us = timeit(lambda: ops.attn_decode(q, kc, vc, bt, sl, out, part, ctr, nh, nkv, D, 64, ch, sc,
                                                    grid_chunks=gc, fused=True))
                best = min(best, us)
                line.append(f"fused c{ch} {us:6.2f}")
            for gc in [16, 32, 64, 128, 256]:
                gc_eff = min(gc, (L + 127) // 128)
                if gc_eff < gc and gc > 16:
                    continue
                part, ctr = ops.decode_attn_workspace(1, nh, nkv, D, gc_eff, "cuda")
                us = timeit(lambda: ops.attn_decode(q, kc, vc, bt, sl, out, part, ctr, nh, nkv, D, 64, 128, sc,
                                                    grid_chunks=gc_eff))
                best = min(best, us)
                line.append(f"split g{gc_eff} {us:6.2f}")
            print(f"attn nh={nh} nkv={nkv} D={D} L={L:6d}: " + "  ".join(line)
                  + f"  | best {gb / best * 1e6 / 1e3:5.2f} TB/s", flush=True)


def bench_attn_oproj(shapes=((32, 8, 128, 4096),), lens=(128, 1024, 2048, 2300, 4096, 6000, 8000, 9000, 12000,
                                                          16000)):
    """Decode attention + o_proj + residual of ONE row per layer: the fused launch (attn_oproj.hip)
    against the engine's two launches (attn_decode in the bucket's form + o GEMV with the residual
    epilogue). Graph-timed over COPIES cycled per call (>= 512 MB of weights and K/V, beyond the
    256 MB Infinity Cache), so every call reads cold weights as a decode step does."""
    from llm_consensus_amd.engine.engine import attn_buckets, split_blocks_per_head
    from llm_consensus_amd.ops import EPI_RESADD

    for nh, nkv, D, H in shapes:
        nc = ops.attn_oproj_grid(H, nh, nkv, D)
        sc = 1 / math.sqrt(D)
        for L in lens:
            cap = 1024
            while cap < L:
                cap *= 2
            chunk = ops.attn_oproj_chunk(cap, nc)
            bk = attn_buckets(cap, split_blocks_per_head(nh, nkv), ops.FUSED_ATTN_MAX_KEYS, nh // nkv, nkv)[-1]
            _, ch2, gc2, fused2 = bk
            w_bytes = H * nh * D * 2
            kv_bytes = L * nkv * D * 4
            copies = max(4, (512 << 20) // (w_bytes + kv_bytes) + 1)
            cases = [_attn_case(L, nh, nkv, D) for _ in range(copies)]
            wos = [(torch.randn(H, nh * D, device="cuda") / math.sqrt(nh * D)).to(BF) for _ in range(copies)]
            h = torch.zeros(1, H, dtype=BF, device="cuda")
            attn = torch.zeros(1, nh * D, dtype=BF, device="cuda")
            ws = ops.attn_oproj_workspace(H, nh, nkv, D, nc, "cuda")
            part, ctr = ops.decode_attn_workspace(1, nh, nkv, D, max(gc2, 32), "cuda")
            fault = torch.zeros(1, dtype=torch.int32, device="cuda")
            fault1 = torch.zeros(1, dtype=torch.int32, device="cuda")
            it = [0]

            def two():
                kc, vc, bt, sl, q, out = cases[it[0] % copies]
                ops.attn_decode(q, kc, vc, bt, sl, out, part, ctr, nh, nkv, D, 64, ch2, sc, grid_chunks=gc2,
                                fused=fused2, fault=fault)
                ops.linear(out, wos[it[0] % copies], EPI_RESADD, out=h)
                it[0] += 1

            def one(mode=0):
                kc, vc, bt, sl, q, out = cases[it[0] % copies]
                ops.attn_oproj(q, kc, vc, bt, sl, wos[it[0] % copies], h, attn, ws, nh, nkv, D, 64, chunk, nc, sc,
                               fault=fault1, mode=mode)
                it[0] += 1

            n = copies * max(1, 48 // copies)
            t2 = timeit(two, iters=n)
            # AO_MODES: comma list of kernel mode bits (attn_oproj.hip llmc_attn_oproj)
            modes = [int(m) for m in os.environ.get("AO_MODES", "0,1,3,7").split(",")]
            tm = [(m, timeit(lambda m=m: one(m), iters=n) if chunk else float("nan")) for m in modes]
            torch.cuda.synchronize()
            print(f"attn+o nh={nh} nkv={nkv} D={D} H={H} L={L:5d} cap={cap}: two launches "
                  f"({'fused' if fused2 else 'split'} c{ch2} g{gc2} + o GEMV) {t2:6.2f} us | one launch "
                  f"(nc {nc}, {chunk} keys/block) " + ", ".join(f"mode {m} {t:6.2f} us" for m, t in tm)
                  + f" | fault {int(fault.item())} / {int(fault1.item())}", flush=True)
            del cases, wos


def bench_attn_batched(shapes=((32, 8, 128),), rows=(1, 4, 16), lens=(2048, 2560, 8192)):
    """Decode attention for B rows per launch (continuous batching): the fused form over the
    engine's bucket (capacity = next power of two >= L, 128/256-key chunks) vs the balanced split
    at several blocks per kv head."""
    for nh, nkv, D in shapes:
        for B in rows:
            for L in lens:
                kc, vc, bt, sl, q, out = _attn_case(L, nh, nkv, D, B=B)
                sc = 1 / math.sqrt(D)
                gb = B * L * nkv * D * 2 * 2 / 1e9
                cap = 1024
                while cap < L:
                    cap *= 2
                line, best = [], 1e9
                for ch in (128, 256):
                    gc = cap // ch
                    part, ctr = ops.decode_attn_workspace(B, nh, nkv, D, gc, "cuda", fused=True)
                    us = timeit(lambda: ops.attn_decode(q, kc, vc, bt, sl, out, part, ctr, nh, nkv, D, 64, ch, sc,
                                                        grid_chunks=gc, fused=True))
                    best = min(best, us)
                    line.append(f"fused c{ch} {us:6.2f}")
                for gc in (2, 4, 8, 16, 32):
                    part, ctr = ops.decode_attn_workspace(B, nh, nkv, D, gc, "cuda")
                    us = timeit(lambda: ops.attn_decode(q, kc, vc, bt, sl, out, part, ctr, nh, nkv, D, 64, 128, sc,
                                                        grid_chunks=gc))
                    best = min(best, us)
                    line.append(f"split g{gc} {us:6.2f}")
                print(f"attn B={B:2d} nh={nh} nkv={nkv} D={D} L={L:6d}: " + "  ".join(line)
                      + f"  | best {gb / best * 1e6 / 1e3:5.2f} TB/s", flush=True)


def bench_gemv():
    for (N, K, epi, norm) in [(6144, 4096, 0, True), (4096, 4096, 2, False), (28672, 4096, 3, True),
                              (4096, 14336, 2, False), (128256, 4096, 1, True)]:
        x = torch.randn(1, K, device="cuda").to(BF)
        W = (torch.randn(N, K, device="cuda") * 0.02).to(BF)
        nw = torch.ones(K, dtype=BF, device="cuda")
        out = torch.zeros(1, N // 2 if epi == 3 else N, dtype=torch.float32 if epi == 1 else BF, device="cuda")
        us = timeit(lambda: ops.gemv(x, W, epi, out=out, norm_w=nw if norm else None))
        print(f"gemv N={N:6d} K={K:5d} epi={epi}: {us:8.2f} us  {N * K * 2 / us / 1e6:6.2f} TB/s")


SWEEP = ["256x1u8", "256x2u4", "256x4u4", "512x1u8", "512x2u4", "128x1u8", "64x1u8", "1024x1u4", "256x1u4",
         "256x2u8", "512x4u2", "128x2u4", "1024x1u8", "1024x2u4", "1024x2u2", "1024x1u2", "768x1u4", "1024x4u2", "1024x1u6",
         "768x2u4", "640x1u8", "896x1u4", "768x2u2", "1024x2u2b"]


ALL_VARIANTS = os.environ.get("SWEEP_ALL") == "1"


def bench_gemv_sweep(shapes=None):
    """GEMV geometry sweep on COLD weights: the graph cycles through enough copies of W to exceed
    the 256 MB MALL, as in a real decode step (16 GB streamed per token)."""
    from llm_consensus_amd.utils.native import kernels

    k = kernels()
    for (N, K) in shapes or [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]:
        if K * 2 > 64 * 1024:
            continue
        copies = max(2, (1 << 30) // (N * K * 2))
        Ws = [(torch.randn(N, K, device="cuda") * 0.02).to(BF) for _ in range(copies)]
        x = torch.randn(1, K, device="cuda").to(BF)
        nw = torch.ones(K, dtype=BF, device="cuda")
        out = torch.zeros(1, N, dtype=BF, device="cuda")
        res = []
        for v, name in enumerate(SWEEP):
            keep = os.environ.get("SWEEP_ONLY")
            if keep:
                if name not in keep.split(","):
                    continue
            elif not ALL_VARIANTS and name not in ("256x2u4", "512x1u8", "1024x1u4", "1024x1u6", "1024x1u8", "768x1u4",
                                                   "1024x1u2"):
                continue
            st = torch.cuda.current_stream().cuda_stream

            def run():
                for W in Ws:
                    k.gemv_sweep(v, x.data_ptr(), nw.data_ptr(), W.data_ptr(), out.data_ptr(), N, K,
                                 torch.cuda.current_stream().cuda_stream)
            us = timeit(run, iters=2, warm=1) / copies
            res.append(f"{name} {us:6.2f}")
        del Ws
        torch.cuda.empty_cache()
        print(f"sweep N={N} K={K} ({N * K * 2 / 1e6:.0f} MB, {copies} copies): " + "  ".join(res), flush=True)


def bench_batched_decode(shapes=None, rows=(1, 2, 3, 4, 5, 8, 12, 16)):
    """Batched decode projections on COLD weights: the dispatcher's form per row count (VALU GEMV
    for M <= 2, MFMA form 3-32) and the MFMA form forced at every M, with the fused norm prologue
    where the layer has one (qkv, gate_up, lm_head) and the residual add elsewhere."""
    from llm_consensus_amd import ops

    for (N, K, epi, norm) in shapes or [(6144, 4096, 0, True), (4096, 4096, 2, False), (28672, 4096, 3, True),
                                        (4096, 14336, 2, False), (128256, 4096, 1, True)]:
        copies = max(2, (1 << 30) // (N * K * 2))
        Ws = [(torch.randn(N, K, device="cuda") * 0.02).to(BF) for _ in range(copies)]
        nw = torch.ones(K, dtype=BF, device="cuda") if norm else None
        line = []
        for M in rows:
            x = torch.randn(M, K, device="cuda").to(BF)
            n_out = N // 2 if epi == 3 else N
            out = torch.zeros(M, n_out, dtype=torch.float32 if epi == 1 else BF, device="cuda")
            t = {}
            for form, fn in (("auto", ops.linear), ("mfma", ops.gemvm)):
                if form == "mfma" and M > 2 and "auto" in t:
                    continue  # the dispatcher already ran the MFMA form

                def run():
                    for W in Ws:
                        fn(x, W, epi, out=out, norm_w=nw)
                t[form] = timeit(run, iters=2, warm=1) / copies
            tbs = N * K * 2 / t["auto"] / 1e6
            extra = f"/{t['mfma']:.2f}" if "mfma" in t else ""
            line.append(f"M={M} {t['auto']:6.2f}{extra} ({tbs:4.2f} TB/s)")
        del Ws
        torch.cuda.empty_cache()
        print(f"batched N={N} K={K} epi={epi}{' +norm' if norm else ''}: " + "  ".join(line), flush=True)


def bench_gemvm_forms(shapes=None, rows=(3, 4, 5, 8, 12, 16)):
    """The MFMA decode form's four variants per shape and row count (cold weights): (row groups per
    wave, x path) = 1: (1, L2)  2: (1, LDS)  3: (2, L2)  4: (2, LDS); 'auto' = the shape rule."""
    from llm_consensus_amd import ops

    for (N, K, epi, norm) in shapes or [(6144, 4096, 0, True), (4096, 4096, 2, False), (28672, 4096, 3, True),
                                        (4096, 14336, 2, False), (128256, 4096, 1, True), (14336, 4096, 3, True)]:
        copies = max(2, (1 << 30) // (N * K * 2))
        Ws = [(torch.randn(N, K, device="cuda") * 0.02).to(BF) for _ in range(copies)]
        nw = torch.ones(K, dtype=BF, device="cuda") if norm else None
        for M in rows:
            x = torch.randn(M, K, device="cuda").to(BF)
            n_out = N // 2 if epi == 3 else N
            out = torch.zeros(M, n_out, dtype=torch.float32 if epi == 1 else BF, device="cuda")
            res = []
            for form in (0, 1, 2, 3, 4) if M <= 16 else (0, 1, 2, 3):  # 17-32 rows: no form 4 (LDS)
                def run():
                    for W in Ws:
                        ops.gemvm(x, W, epi, out=out, norm_w=nw, form=form)
                res.append(f"{'auto' if form == 0 else form}:{timeit(run, iters=2, warm=1) / copies:6.2f}")
            print(f"forms N={N} K={K} epi={epi} M={M}: " + "  ".join(res), flush=True)
        del Ws
        torch.cuda.empty_cache()


def bench_qkv_rope():
    """qkv GEMV with the RoPE + paged-KV-write epilogue vs the same GEMV with a plain bf16
    epilogue (both with the fused RMSNorm prologue), cold weights: what the epilogue costs."""
    from llm_consensus_amd.ops import oracle

    for (nh, nkv, D, H) in [(32, 8, 128, 4096), (32, 32, 96, 3072), (4, 1, 128, 4096)]:
        N = (nh + 2 * nkv) * D
        copies = max(2, (1 << 30) // (N * H * 2))
        Ws = [(torch.randn(N, H, device="cuda") * 0.02).to(BF) for _ in range(copies)]
        x = torch.randn(1, H, device="cuda").to(BF)
        nw = torch.ones(H, dtype=BF, device="cuda")
        bs, nb = 64, 64
        kc = torch.zeros(nb, nkv, bs, D, dtype=BF, device="cuda")
        vc = torch.zeros_like(kc)
        cos_t, sin_t = oracle.rope_tables([1.0 / (10000 ** (2 * i / D)) for i in range(D // 2)], 4096)
        cos_t, sin_t = cos_t.cuda(), sin_t.cuda()
        pos = torch.tensor([1000], dtype=torch.int32, device="cuda")
        slots = torch.tensor([1000], dtype=torch.int32, device="cuda")
        q = torch.zeros(1, nh * D, dtype=BF, device="cuda")
        out = torch.zeros(1, N, dtype=BF, device="cuda")

        def rope():
            for W in Ws:
                ops.qkv_rope(x, W, nw, 1e-5, q, kc, vc, pos, slots, cos_t, sin_t, nh, nkv, D, bs)

        def plain():
            for W in Ws:
                ops.gemv(x, W, 0, out=out, norm_w=nw)

        def bare():
            for W in Ws:
                ops.gemv(x, W, 0, out=out)
        tr = timeit(rope, iters=2, warm=1) / copies
        tp = timeit(plain, iters=2, warm=1) / copies
        tb = timeit(bare, iters=2, warm=1) / copies
        print(f"qkv nh={nh} nkv={nkv} D={D} H={H} (N={N}, {N * H * 2 / 1e6:.1f} MB): rope+kv epilogue {tr:6.2f} us, "
              f"plain (norm prologue) {tp:6.2f} us, bare (no norm) {tb:6.2f} us", flush=True)


def bench_launch():
    x = torch.zeros(1, 4096, dtype=BF, device="cuda")
    w = torch.ones(4096, dtype=BF, device="cuda")
    us = timeit(lambda: ops.rmsnorm(x, w, 1e-5, out=x))
    print(f"rmsnorm [1,4096] (launch-bound floor): {us:.2f} us")


def bench_prefill():
    """Prefill GEMM (ours vs torch.matmul = hipBLASLt) and flash prefill attention throughput."""
    for (M, N, K) in [(8192, 28672, 4096), (8192, 6144, 4096), (8192, 4096, 4096), (8192, 4096, 14336),
                      (13463, 28672, 4096), (2048, 6144, 4096),
                      # Llama-3-70B TP=4 rank (config 5 judge prefill): qkv, o, gate_up, down
                      (8192, 2560, 8192), (8192, 8192, 2048), (8192, 14336, 8192), (8192, 8192, 7168),
                      # Llama-3-8B TP=8 rank (the N=8 bench judge): qkv, gate_up, down
                      (8192, 768, 4096), (8192, 3584, 4096), (8192, 4096, 1792),
                      # the TP=8 rank's qkv on the 33k-token judge prompt and a 2k prompt
                      (33000, 768, 4096), (2048, 768, 4096)]:
        if os.environ.get("GEMM_CASES") and f"{M},{N},{K}" not in os.environ["GEMM_CASES"].split(";"):
            continue
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(BF)  # full-range random data (guide rule 25)
        W = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(BF)
        out = torch.empty(M, N, dtype=BF, device="cuda")
        t_ours = timeit(lambda: ops.gemm(x, W, 0, out=out), iters=10)
        t_128 = timeit(lambda: ops.gemm128(x, W, 0, out=out), iters=10)
        t_nar = timeit(lambda: ops.gemm_narrow(x, W, 0, out=out), iters=10)
        t_ref = timeit(lambda: torch.matmul(x, W.t(), out=out), iters=10)  # hipBLASLt: reference only
        fl = 2 * M * N * K
        line = (f"gemm M={M} N={N} K={K}: ours {t_ours:8.1f} us {fl / t_ours / 1e6:6.0f} TF/s | 128x128 {t_128:8.1f} us "
                f"{fl / t_128 / 1e6:6.0f} TF/s | 128x192 {t_nar:8.1f} us {fl / t_nar / 1e6:6.0f} TF/s | "
                f"torch {t_ref:8.1f} us {fl / t_ref / 1e6:6.0f} TF/s")
        print(line, flush=True)
    bench_attn_prefill()


def bench_attn_prefill(cases=((32, 8, 2048, 2048), (32, 8, 8192, 8192), (32, 8, 8192, 32768), (32, 8, 2304, 9000),
                              (4, 1, 8192, 8192), (4, 1, 8192, 32768), (16, 2, 8192, 8192))):
    """Causal flash prefill (attn_prefill.hip) on (heads, kv heads, T new tokens, ctx keys): Llama-3-8B
    and its TP=8 rank (4 heads on 1 kv head), Llama-3-70B TP=4 rank (16 on 2)."""
    D, bs = 128, 64
    if os.environ.get("PF_CASES"):  # "nh,nkv,T,ctx;..."
        cases = [tuple(int(x) for x in c.split(",")) for c in os.environ["PF_CASES"].split(";")]
    for (nh, nkv, T, ctx) in cases:
        nb = (ctx + bs - 1) // bs + 1
        kc = torch.randn(nb, nkv, bs, D, device="cuda").to(BF)
        vc = torch.randn_like(kc)
        bt = torch.arange(nb, dtype=torch.int32, device="cuda").view(1, -1)
        q = torch.randn(T, nh * D, device="cuda").to(BF)
        out = torch.empty_like(q)
        qs = torch.tensor([0], dtype=torch.int32, device="cuda")
        ql = torch.tensor([T], dtype=torch.int32, device="cuda")
        cl = torch.tensor([ctx], dtype=torch.int32, device="cuda")
        # causal FLOPs of the last T queries over ctx keys
        fl = 4 * nh * D * (T * ctx - T * (T - 1) / 2)
        plan = ops.attn_prefill_plan(1, T, ctx, nh, nkv, ksplit=-1)
        ws = ops.attn_prefill_workspace(4, T, nh, D, "cuda", 1, nkv, T)
        res = []
        # one throwaway timing first: the first measurement of a shape ran ~7 % slow (clock ramp)
        timeit(lambda: ops.attn_prefill(q, kc, vc, bt, qs, ql, cl, out, T, nh, nkv, D, bs, 1 / math.sqrt(D),
                                        max_ctx=ctx, ksplit=1, ws=ws), iters=3)
        extra = [tuple(int(x) for x in c.split(",")) for c in os.environ.get("PF_SPLITS", "").split(";") if c]
        for k, km in dict.fromkeys([plan, (1, 1), (2, 8), (2, 16), (4, 4), (4, 8), (4, 16)] + extra):
            us = timeit(lambda: ops.attn_prefill(q, kc, vc, bt, qs, ql, cl, out, T, nh, nkv, D, bs, 1 / math.sqrt(D),
                                                 max_ctx=ctx, ksplit=k, kmin=km, ws=ws), iters=3)
            tag = "plan" if (k, km) == plan else ""
            res.append(f"{tag}({k},{km if k > 1 else '-'}) {us:7.1f} us {fl / us / 1e6:4.0f} TF/s")
        print(f"attn_prefill nh={nh} nkv={nkv} T={T} ctx={ctx}: " + " | ".join(res), flush=True)


def bench_moe(tokens=(2048, 8192, 16384)):
    """Mixtral-8x7B grouped expert GEMMs (top-2 of 8, hidden 4096, FFN 14336), routed by random
    router logits: gate_up (SiLU-mul epilogue) and down over moe_align's list; TF/s on the routed
    pairs' FLOPs (padding rows excluded)."""
    E, k, H, I = 8, 2, 4096, 14336
    wgu = ((torch.rand(E, 2 * I, H, device="cuda") * 2 - 1) * 0.05).to(BF)
    wd = ((torch.rand(E, H, I, device="cuda") * 2 - 1) * 0.05).to(BF)
    for T in tokens:
        x = (torch.rand(T, H, device="cuda") * 2 - 1).to(BF)
        w = torch.empty(T, k, device="cuda")
        ids = torch.empty(T, k, dtype=torch.int32, device="cuda")
        ops.moe_route(torch.randn(T, E, device="cuda"), k, w, ids)
        tile = ops.moe_tile(T * k, E)
        mt = ops.moe_max_tiles(T * k, E, tile)
        sr = torch.empty(mt * tile, dtype=torch.int32, device="cuda")
        te = torch.empty(mt, dtype=torch.int32, device="cuda")
        tc = torch.empty(1, dtype=torch.int32, device="cuda")
        ops.moe_align(ids, E, sr, te, tc, tile=tile)
        act = torch.empty(T * k, I, dtype=BF, device="cuda")
        y = torch.empty(T * k, H, dtype=BF, device="cuda")
        t_gu = timeit(lambda: ops.moe_gemm(x, wgu, sr, te, tc, act, 2 * I, H, mt, k, epi=ops.EPI_SILU, tile=tile),
                      iters=10)
        t_dn = timeit(lambda: ops.moe_gemm(act, wd, sr, te, tc, y, H, I, mt, 1, tile=tile), iters=10)
        f_gu, f_dn = 2 * T * k * 2 * I * H, 2 * T * k * H * I
        print(f"moe T={T} tile={tile}: gate_up+silu {t_gu:8.1f} us {f_gu / t_gu / 1e6:6.0f} TF/s | down {t_dn:8.1f} us "
              f"{f_dn / t_dn / 1e6:6.0f} TF/s", flush=True)


def bench_attn_rows_policy(rows=(1, 2, 4, 8, 16, 32), lens=(700, 2560, 8192, 13500)):
    """Batching engines' decode attention: the grid a batch-invariant policy can use. 'rowsN' = the
    balanced split at max(1, 256 / (N x nkv)) blocks per kv head for an engine sized for N rows
    (every B); 'mcK' = the split with a K-key minimum per block over min(32, capacity / K) blocks
    per head for the power-of-two bucket capacity (a row's partition then depends on its own
    length only). us per launch."""
    nh, nkv, D = 32, 8, 128
    sc = 1 / math.sqrt(D)
    for L in lens:
        for B in rows:
            kc, vc, bt, sl, q, out = _attn_case(L, nh, nkv, D, B=B)
            line = []
            for eng_rows in (16, 32):
                gc = max(1, 256 // (eng_rows * nkv))
                part, ctr = ops.decode_attn_workspace(B, nh, nkv, D, gc, "cuda")
                us = timeit(lambda: ops.attn_decode(q, kc, vc, bt, sl, out, part, ctr, nh, nkv, D, 64, 128, sc,
                                                    grid_chunks=gc))
                line.append(f"rows{eng_rows}(g{gc}) {us:7.2f}")
            cap = 1024
            while cap < L:
                cap *= 2
            for mc in (512, 1024, 2048):
                gc = min(32, -(-cap // mc))  # the bucket's grid: no block beyond the capacity
                part, ctr = ops.decode_attn_workspace(B, nh, nkv, D, gc, "cuda")
                us = timeit(lambda: ops.attn_decode(q, kc, vc, bt, sl, out, part, ctr, nh, nkv, D, 64, mc, sc,
                                                    grid_chunks=gc))
                line.append(f"mc{mc}(g{gc}) {us:7.2f}")
            print(f"attn-rows L={L:6d} B={B:2d}: " + "  ".join(line), flush=True)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("launch", "all"):
        bench_launch()
    if what in ("attn", "all"):
        bench_attn()
    if what in ("attn-phi3",):  # Phi-3-mini: 32 heads = 32 kv heads, D = 96
        bench_attn(((32, 32, 96),))
    if what in ("attn-tp",):  # TP ranks' shapes only (G = 8 / 4 on one or two kv heads)
        bench_attn(((16, 2, 128), (8, 1, 128), (4, 1, 128)))
    if what in ("gemv", "all"):
        bench_gemv()
    if what in ("sweep",):
        bench_gemv_sweep()
    if what in ("sweep-phi3",):  # Phi-3-mini shapes (K = 3072 / 8192)
        bench_gemv_sweep([(9216, 3072), (16384, 3072), (3072, 3072), (3072, 8192)])
    if what in ("sweep-tp8",):  # one TP=8 rank of Llama-3-8B: qkv, gate_up, o, down
        bench_gemv_sweep([(768, 4096), (1536, 4096), (3584, 4096), (4096, 512), (4096, 1792)])
    if what in ("sweep-70b-tp4",):  # one TP=4 rank of Llama-3-70B: qkv, gate_up, o, down
        bench_gemv_sweep([(2560, 8192), (14336, 8192), (8192, 2048), (8192, 7168)])
    if what in ("attn-oproj",):  # fused decode attention + o_proj (one row) vs the two launches
        bench_attn_oproj()
    if what in ("attn-batched",):  # decode attention with many rows per launch
        bench_attn_batched()
    if what in ("gemvm-forms",):  # the MFMA decode form's variants
        bench_gemvm_forms()
    if what in ("batched",):  # decode projections at continuous-batching row counts
        bench_batched_decode()
    if what in ("attn-rows",):  # batching engines' attention grid policy
        bench_attn_rows_policy()
    if what in ("batched32",):  # two 16-token column groups (17-32 rows) against 16
        bench_batched_decode(rows=(8, 16, 17, 24, 32))
        bench_gemvm_forms(rows=(24, 32))
    if what in ("qkv-rope",):
        bench_qkv_rope()
    if what in ("moe",):  # Mixtral grouped expert GEMMs
        bench_moe()
    if what in ("attn-prefill",):
        bench_attn_prefill()
    if what in ("prefill",):
        bench_prefill()
