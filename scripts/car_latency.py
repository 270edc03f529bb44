"""Latency of the custom one-shot all-reduce (K13) for a decode-sized message, measured with W rank
processes sharing ONE GPU (the IPC/flag protocol of the xGMI path without the link): each rank
captures 200 all-reduces of a [1, 4096] bf16 hidden row in a HIP graph and times its replays.
A lower bound for the per-all-reduce cost of a TP decode step (64 per token for Llama-3-8B).

  python scripts/car_latency.py --world 2,4
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _worker(rank, world, port, n, reps, q):
    import torch.distributed as dist

    from llm_consensus_amd.parallel.comm import TPGroup

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    tp = TPGroup(dist.group.WORLD, rank, world)
    tp.enable_custom("cuda:0", cap=1 << 20)
    x = torch.randn(n, device="cuda").to(torch.bfloat16)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(4):
            tp.all_reduce_(x)
    torch.cuda.synchronize()
    dist.barrier()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            tp.all_reduce_(x)
    dist.barrier()
    times = []
    for _ in range(5):
        torch.cuda.synchronize()
        dist.barrier()
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
    q.put((rank, min(times) / reps * 1e6, tp.custom.timed_out()))
    dist.barrier()
    tp.custom.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", default="2,4")
    ap.add_argument("--elems", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    for w in [int(x) for x in a.world.split(",")]:
        q = ctx.Queue()
        port = 29700 + w
        ps = [ctx.Process(target=_worker, args=(r, w, port, a.elems, a.reps, q)) for r in range(w)]
        for p in ps:
            p.start()
        res = sorted(q.get(timeout=300) for _ in ps)
        for p in ps:
            p.join(timeout=60)
        us = max(r[1] for r in res)
        print(f"custom all-reduce, {w} ranks on one GPU, {a.elems} bf16: {us:.2f} us per all-reduce "
              f"(graph-replayed, max over ranks; timed out: {any(r[2] for r in res)})", flush=True)


if __name__ == "__main__":
    main()
