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


def kv_rows(e, seq, layer, n=None, cache=None):
    bs = e.bs
    c = e.k_cache if cache is None else cache
    rows = [c[layer, seq.blocks[p // bs], :, p % bs].float().cpu() for p in range(n or len(P))]
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
    e.free_sequence(s)
    wsum = sum(float(L.w_gu.float().sum()) + float(L.w_down.float().sum()) for L in e.w.layers if L.w_gu is not None)
    gen = e.generate_ids(P, 12, temperature=0.0, stop_on_eos=False)
    wsum2 = sum(float(L.w_gu.float().sum()) + float(L.w_down.float().sum()) for L in e.w.layers if L.w_gu is not None)
    if os.environ.get("DBG_KV_AFTER"):  # prefill + greedy decode on a kept sequence: K and V rows
        from llm_consensus_amd.engine import SamplingParams
        s2 = e.new_sequence()
        e.prefill([s2], [P])
        g2 = e.decode([s2], [SamplingParams(2, 0.0, 1.0, 0, 0, False)])[0]
        torch.cuda.synchronize()
        lg = e.logits[0].float().cpu()
        # teacher-forced: prefill P + [first token] on a fresh sequence, full logits of the last row
        s3 = e.new_sequence()
        e.prefill([s3], [P + g2[:1]])
        lt = e.full_logits(s3).float().cpu()
        print(f"rank {rank} decode-step logits vs teacher-forced prefill: max err {float((lg - lt).abs().max()):.4f}"
              f" argmax {int(lg.argmax())} vs {int(lt.argmax())}", flush=True)
        kv = [(kv_rows(e, s2, li, len(P) + 5).tolist(), kv_rows(e, s2, li, len(P) + 5, e.v_cache).tolist())
              for li in range(e.cfg.n_layers)]
        torch.save({"gen": g2, "kv": kv}, f"gpurun_out/kv_{os.environ.get('DBG_TAG', 'x')}_r{rank}.pt")
    if os.environ.get("DBG_NOSP_AFTER"):
        e.ecfg.sequence_parallel = False  # (c): decode after a non-SP prefill, state left by the SP one
        gen = e.generate_ids(P, 12, temperature=0.0, stop_on_eos=False)
    print(f"rank {rank} weights {wsum} -> {wsum2} gen {gen} timed_out {e.tp.custom.timed_out()}", flush=True)
    if rank == 0:
        q.put(([o.tolist() for o in out], gen))
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
    ref.free_sequence(s)
    print("ref gen", ref.generate_ids(P, 12, temperature=0.0, stop_on_eos=False), flush=True)
    cfgs = [{}, {"expert_parallel": True}, {"expert_parallel": True, "sp_min_tokens": 16}, {"sp_min_tokens": 16},
            {"expert_parallel": True, "sp_min_tokens": 16, "use_graphs": False},
            {"expert_parallel": True, "use_graphs": False, "steps_per_graph": 1},
            {"expert_parallel": True, "sp_min_tokens": 16, "use_graphs": False, "steps_per_graph": 1}]
    only = os.environ.get("DBG_ONLY")
    for i, ekw in enumerate(cfgs):
        if only and str(i) not in only.split(","):
            continue
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=w, args=(r, 2, 29700 + i, ekw, q)) for r in range(2)]
        [p.start() for p in ps]
        out, gen = q.get(timeout=200)
        print(ekw, "gen", gen, flush=True)
        [p.join() for p in ps]
        for li, o in enumerate(out):
            o = torch.tensor(o)
            r = refs[li][:, : o.shape[1]]
            err = (o - r).abs().amax(dim=(1, 2))
            print(ekw, "layer", li, "max err", round(err.max().item(), 4), "worst rows", err.topk(3).indices.tolist(),
                  flush=True)
