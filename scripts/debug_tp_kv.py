"""Debug harness: KV cache rows written by a TP=2 prefill (ranks sharing one GPU, gloo) vs the
TP=1 engine, per engine config (SP / EP variants). Prints per-layer max error of rank 0's heads."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
P = [(i * 13) % 700 + 256 for i in range(40)]
NAME = os.environ.get("DBG_MODEL", "mixtral-tiny")


def kv_rows(e, seq, layer):
    bs = e.bs
    rows = [e.k_cache[layer, seq.blocks[p // bs], :, p % bs].float().cpu() for p in range(len(P))]
    return torch.stack(rows)  # [T, nkv, D]


def w(rank, world, port, ekw, q):
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.models.config import FAMILIES
    from llm_consensus_amd.parallel.comm import TPGroup

    tp = TPGroup(dist.group.WORLD, rank, world)
    tp.enable_custom("cuda:0")
    e = Engine(FAMILIES[NAME], EngineConfig(device="cuda:0", max_context=256, seed=5, **ekw), tp=tp)
    s = e.new_sequence()
    e.prefill([s], [P])
    torch.cuda.synchronize()
    out = [kv_rows(e, s, li) for li in range(e.cfg.n_layers)]
    if rank == 0:
        q.put([o.tolist() for o in out])
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.models.config import FAMILIES

    ref = Engine(FAMILIES[NAME], EngineConfig(device="cuda:0", max_context=256, seed=5))
    s = ref.new_sequence()
    ref.prefill([s], [P])
    torch.cuda.synchronize()
    refs = [kv_rows(ref, s, li) for li in range(ref.cfg.n_layers)]
    for i, ekw in enumerate([{}, {"expert_parallel": True}, {"expert_parallel": True, "sp_min_tokens": 16},
                             {"sp_min_tokens": 16}]):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=w, args=(r, 2, 29700 + i, ekw, q)) for r in range(2)]
        [p.start() for p in ps]
        out = q.get(timeout=200)
        [p.join() for p in ps]
        for li, o in enumerate(out):
            o = torch.tensor(o)
            r = refs[li][:, : o.shape[1]]
            err = (o - r).abs().amax(dim=(1, 2))
            print(ekw, "layer", li, "max err", round(err.max().item(), 4), "worst rows", err.topk(3).indices.tolist(),
                  flush=True)
