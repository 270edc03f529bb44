"""Tensor-parallel decode of a real TP group rehearsed on ONE GPU: W rank processes share the card,
each engine stream restricted to its own 256 / W CUs (``EngineConfig.cu_mask``), so ranks that
spin on each other (the custom collectives, the fused all-reduce epilogue) run side by side as on
separate GPUs instead of time-sharing CUs. Every rank holds the shard a ``--shape-tp``-way TP rank
of the model holds (heads, kv heads, FFN rows and vocab divided by shape-tp) and the group's
collectives are the real ones over ``--world`` ranks ([1, hidden] bf16 all-reduces, the logits
all-gather), so a --shape-tp 8 --world 2 run is the decode chain of a TP=8 judge rank with its
64 all-reduces per token, at half the chip per rank and HBM shared by the two ranks.

  python scripts/tp_rehearsal.py --shape-tp 8 --world 2 --ctx 2048 --tokens 256 [--fused-ar 0|1]
"""
import argparse
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker(rank, a, port, q):
    total = 256
    per = total // a.world
    os.environ["LLMC_CU_MASK"] = f"{rank * per}-{(rank + 1) * per - 1}" if a.cu_mask else ""
    # ranks share the GPU: the fused all-reduce only runs when forced (each rank has its own CUs here)
    os.environ["LLMC_FUSED_AR"] = "force" if a.fused_ar else "0"
    import torch
    import torch.distributed as dist

    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.models.config import FAMILIES
    from llm_consensus_amd.parallel.comm import TPGroup

    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=a.world)
        base = FAMILIES[a.model]
        k = a.shape_tp // a.world  # the engine divides by world: each rank ends up with 1 / shape_tp
        cfg = base.with_(name=f"{a.model}-tp{a.shape_tp}-rehearsal", n_heads=base.n_heads // k,
                         n_kv_heads=base.n_kv_heads // k, intermediate=base.intermediate // k, vocab=base.vocab // k)
        tp = TPGroup(dist.group.WORLD, rank, a.world, ctrl=dist.group.WORLD)
        ok = tp.enable_custom("cuda:0")
        e = Engine(cfg, EngineConfig(device="cuda:0", max_context=a.ctx + a.tokens + 64, seed=1), tp=tp)
        e.warmup_graphs()
        prompt = [(i * 7919) % (cfg.vocab - 512) + 256 for i in range(a.ctx)]
        e.generate_ids(prompt[:64], 16, stop_on_eos=False)  # warm
        res = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            dist.barrier()
            t = time.perf_counter()
            out = e.generate_ids(prompt, a.tokens, stop_on_eos=False)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            s = e.new_sequence()
            dist.barrier()
            t = time.perf_counter()
            e.prefill([s], [prompt])
            torch.cuda.synchronize()
            tp_s = time.perf_counter() - t
            e.free_sequence(s)
            res.append(1000 * (dt - tp_s) / len(out))
        kcount = None
        if a.trace_kernels:  # the decode's kernels by name (torch.profiler / roctracer), 32 tokens
            from torch.profiler import ProfilerActivity, profile

            torch.cuda.synchronize()
            dist.barrier()
            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                e.generate_ids(prompt[:64], 32, stop_on_eos=False)
                torch.cuda.synchronize()
            kcount = {}
            for ev in prof.key_averages():
                if ev.device_type.name == "CUDA" or "CUDA" in str(ev.device_type):
                    kcount[ev.key] = kcount.get(ev.key, 0) + ev.count
        q.put((rank, ok, tp.custom_fused is not None, min(res), tp.custom_timed_out(), kcount))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put((rank, False, False, repr(ex) + traceback.format_exc(), True, None))


def main():
    import torch.multiprocessing as mp

    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--shape-tp", type=int, default=8)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--ctx", type=int, default=2048)
    ap.add_argument("--tokens", type=int, default=256)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--fused-ar", type=int, default=1)
    ap.add_argument("--cu-mask", type=int, default=1, help="0: ranks time-share every CU")
    ap.add_argument("--trace-kernels", type=int, default=0,
                    help="1: rank 0 lists the kernels of 32 decode tokens (prefill of 64 included) by name")
    a = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, a, port, q)) for r in range(a.world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=900) for _ in range(a.world))
    for p in procs:
        p.join(timeout=60)
    for rank, ok, fused, ms, tmo, _ in res:
        if isinstance(ms, str):
            print(f"rank {rank} failed: {ms}", flush=True)
            sys.exit(1)
    worst = max(r[3] for r in res)
    print(f"{a.model} shape TP={a.shape_tp} over {a.world} ranks (cu_mask={a.cu_mask}, custom={res[0][1]}, "
          f"fused_ar={res[0][2]}) ctx={a.ctx}: decode {worst:.3f} ms/token (ranks {[round(r[3], 3) for r in res]}), "
          f"timed_out={any(r[4] for r in res)}", flush=True)
    if res[0][5]:
        print("rank 0 kernels over 32 decode tokens (+ a 64-token prefill), launches by name:", flush=True)
        for name, n in sorted(res[0][5].items(), key=lambda kv: -kv[1])[:25]:
            print(f"  {n:6d}  {name[:110]}", flush=True)
        car = sum(n for k, n in res[0][5].items() if "car_" in k)
        print(f"standalone custom all-reduce / all-gather launches (car_*): {car}", flush=True)


if __name__ == "__main__":
    main()
