"""Expert-parallel prefill of a Mixtral-shaped MoE over 2 ranks sharing ONE GPU (gloo collectives),
for a kernel trace: the sequence-parallel expert dispatch
(engine ``_moe_ep_a2a``: ``moe_ep_dispatch`` -> ``gather_rows`` -> all-to-all -> grouped expert
GEMMs -> all-to-all -> ``moe_combine`` through the pair slots) and the replicated-token EP path must
run on the llmc kernels only, with no torch sort / bincount / nonzero / index kernels and no host
sync inside the layer loop.

  python3 scripts/ep_prefill_trace.py          (both ranks spawned here)
  bash scripts/prof_ep.sh <tag>                 (each rank under its own rocprofv3)
"""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker(rank, world, port, tokens):
    import torch
    import torch.distributed as dist

    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.models.config import FAMILIES
    from llm_consensus_amd.parallel.comm import TPGroup

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    # Mixtral's layer shape (8 experts, top-2, hidden 4096, FFN 14336) at 4 layers and a small vocab
    cfg = FAMILIES["mixtral-8x7b"].with_(name="mixtral-4l", n_layers=4, vocab=32000)
    # gloo collectives (host bounce) only: no IPC-mapped buffers, so nothing of ours outlives the
    # process's teardown under the profiler
    tp = TPGroup(dist.group.WORLD, rank, world)
    for sp in (True, False):
        e = Engine(cfg, EngineConfig(device="cuda:0", max_context=tokens + 64, seed=3, expert_parallel=True,
                                     sequence_parallel=sp, sp_min_tokens=64, use_graphs=False), tp=tp)
        prompt = [(i * 7919) % 30000 + 256 for i in range(tokens)]
        for _ in range(2):
            s = e.new_sequence()
            e.prefill([s], [prompt])
            torch.cuda.synchronize()
            e.free_sequence(s)
        if rank == 0:
            print(f"EP prefill ({'sequence parallel: all-to-all dispatch' if sp else 'replicated tokens'}) "
                  f"{tokens} tokens x {cfg.n_layers} layers over {world} ranks: ok", flush=True)
        del e
        torch.cuda.empty_cache()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    if "EP_RANK" in os.environ:  # one rank per process (scripts/prof_ep.sh: one profiler per rank)
        _worker(int(os.environ["EP_RANK"]), 2, int(os.environ["EP_PORT"]), 2048)
        sys.exit(0)
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_worker, args=(r, 2, port, 2048)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=600)
    sys.exit(max(abs(p.exitcode or 0) for p in ps))
