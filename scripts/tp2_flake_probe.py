"""Repeat the 2-rank (one GPU, gloo bootstrap) TP=2 vs TP=1 prefill-logits comparison of
tests/test_tp_gpu.py and print, per run, how many logits are off and where (flake hunting).

  python scripts/tp2_flake_probe.py [runs]
"""
import multiprocessing as mp
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

import test_tp_gpu as T  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.models.config import FAMILIES

    ref = Engine(FAMILIES["llama-small"], EngineConfig(device="cuda:0", max_context=512, seed=5))
    s = ref.new_sequence()
    ref.prefill([s], [T.PROMPT])
    ref_logits = ref.full_logits(s).float().cpu()
    ref.free_sequence(s)
    del ref
    torch.cuda.empty_cache()
    cfgs = [("default", {}, {}), ("sp16", {"sp_min_tokens": 16}, {}),
            ("ao-sep", {"_expect_ao": True}, {"LLMC_FUSED_AR": "0", "LLMC_ATTN_OPROJ": "all", "LLMC_TP_ATTN_OPROJ": "1"})]
    ctx = mp.get_context("spawn")
    for it in range(runs):
        for name, ekw, env in cfgs:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            q = ctx.Queue()
            port = T._free_port()
            procs = [ctx.Process(target=T._worker, args=(r, 2, port, "llama-small", q, dict(ekw))) for r in range(2)]
            for p in procs:
                p.start()
            logits, gen, tmo = q.get(timeout=400)
            for p in procs:
                p.join(timeout=120)
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            if isinstance(logits, str):
                print(f"run {it} {name}: worker error {logits[:300]}", flush=True)
                continue
            d = (torch.tensor(logits) - ref_logits).abs()
            bad = (d > 0.05 * ref_logits.abs().max()).nonzero().flatten().tolist()
            print(f"run {it} {name}: max err {d.max().item():.4f}, bad {len(bad)} "
                  f"(first {bad[:8]}, last {bad[-4:]}), timed_out {tmo}", flush=True)


if __name__ == "__main__":
    main()
