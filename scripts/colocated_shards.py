"""Decode throughput of K engines sharing ONE GPU, each holding a TP=--tp shard of Llama-3-8B (heads,
kv heads, FFN rows and vocab divided by tp; no collectives): what a GPU of the N-GPU bench does when
it hosts K model shards at once. K=3 tp=1 is the bench's one-GPU responder phase; K=1 tp=1 a GPU of
the 8-GPU run (one whole responder per GPU); K=2 tp=2 the same GPU if every responder ran
tensor-parallel over a pair of GPUs (two half-models per GPU) — the compute side of that placement,
without its all-reduces.

Each rank process prefills its prompt, waits on a barrier, then decodes --tokens tokens; reported:
every rank's ms/token and the GPU's aggregate weight-streaming rate.

  python scripts/colocated_shards.py --tp 2 --k 2 --ctx 2048 --tokens 512
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker(rank, a, barrier, q):
    import torch

    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.engine.engine import SamplingParams
    from llm_consensus_amd.models.config import FAMILIES

    try:
        torch.cuda.set_device(0)
        base = FAMILIES[a.model]
        tp = a.tp
        cfg = base.with_(name=f"{a.model}-tp{tp}-shard{rank}", n_heads=base.n_heads // tp,
                         n_kv_heads=base.n_kv_heads // tp, intermediate=base.intermediate // tp,
                         vocab=base.vocab // tp)
        e = Engine(cfg, EngineConfig(device="cuda:0", max_context=a.ctx + a.tokens + 64, seed=1 + rank))
        e.warmup_graphs()
        prompt = [(i * 7919 + rank) % (cfg.vocab - 512) + 256 for i in range(a.ctx)]
        e.generate_ids(prompt[:64], 16, stop_on_eos=False)  # warm
        s = e.new_sequence()
        e.prefill([s], [prompt])
        torch.cuda.synchronize()
        barrier.wait()
        t = time.perf_counter()
        out = e.decode([s], [SamplingParams(max_tokens=a.tokens, stop_on_eos=False)])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        e.free_sequence(s)
        q.put((rank, 1000 * dt / len(out[0]), cfg.active_weight_bytes()))
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put((rank, repr(ex) + traceback.format_exc(), 0))
        try:
            barrier.abort()
        except Exception:  # noqa: BLE001
            pass


def main():
    import torch.multiprocessing as mp

    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--k", type=int, default=1, help="engines sharing the GPU")
    ap.add_argument("--ctx", type=int, default=2048)
    ap.add_argument("--tokens", type=int, default=512)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    barrier = ctx.Barrier(a.k)
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, a, barrier, q)) for r in range(a.k)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=900) for _ in range(a.k))
    for p in procs:
        p.join(timeout=60)
    for rank, ms, _ in res:
        if isinstance(ms, str):
            print(f"rank {rank} failed: {ms}", flush=True)
            sys.exit(1)
    worst = max(r[1] for r in res)
    gb = sum(r[2] for r in res) / 1e9
    print(f"{a.model} {a.k} x tp={a.tp} shard(s) on one GPU, ctx {a.ctx}: ms/token {[round(r[1], 3) for r in res]} "
          f"-> {gb:.1f} GB of weights per step of all shards, {gb / worst:.2f} TB/s aggregate", flush=True)


if __name__ == "__main__":
    main()
