#!/usr/bin/env python3
"""Consensus-round benchmark (BASELINE.json metric: p50 end-to-end consensus latency + aggregate
output tokens/sec, N-model fan-out), configs 2/3 generalised to N GPUs:

  * one process per GPU (torchrun; RCCL over xGMI for the gather), weak scaling:
    each GPU hosts ``--models-per-gpu`` Llama-3-8B responders (distinct random-init replicas,
    ``llama-3-8b@<i>``), so an N-GPU run is an (N x models-per-gpu)-model fan-out;
  * the Llama-3-8B judge time-shares the responders' GPUs on its own hipStream(s): by default
    it is tensor-parallel over the first ``--judge-tp`` ranks (auto = every rank whose count
    divides the judge's heads/vocab), so the judge phase — which the reference's semantics make
    strictly sequential after the fan-out (cmd/llm-consensus/main.go:132 then :161) — uses the
    HBM bandwidth of every GPU that just went idle instead of one: TP shards with RCCL for
    prefill-sized all-reduces and the custom one-shot xGMI all-reduce/all-gather inside the
    captured decode graphs. ``--judge-tp 1`` keeps it on GPU 0 only (config 3 as written);
  * one timed step = one full consensus round exactly as ``llm-consensus`` runs it: every
    responder prefills the prompt and decodes ``--max-tokens`` tokens, the responses are
    gathered to rank 0, the judge prompt is rendered with the reference template
    (internal/consensus/judge.go) and the judge prefills it and decodes ``--max-tokens`` tokens
    (a single response is passed through without a judge call, judge.go:74-79).

Reported ``value`` = total generated tokens (responders + judge) per second of wall time over
the whole job; ``ms_per_step`` = mean end-to-end round latency; p50 is in ``extra``.
Data: synthetic prompt (seeded synthetic-tokenizer text), random-init weights, bf16.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def log(*a):
    print(f"[bench r{os.environ.get('RANK', '0')}]", *a, file=sys.stderr, flush=True)


def judge_tp_degree(cfg, world: int, requested: int) -> int:
    """TP degree of the bench judge: ``requested`` if > 0, else the largest t <= min(world, 8)
    that shards the judge's heads, kv heads, FFN and vocab evenly (8 = custom all-reduce limit)."""
    if requested > 0:
        return requested
    for t in range(min(world, 8), 0, -1):
        if not (cfg.n_heads % t or cfg.n_kv_heads % t or cfg.intermediate % t or cfg.vocab % t):
            return t
    return 1


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--judge", default="llama-3-8b")
    ap.add_argument("--models-per-gpu", type=int, default=1)
    ap.add_argument("--max-tokens", type=int, default=4096)
    ap.add_argument("--judge-max-tokens", type=int, default=0, help="0 = same as --max-tokens")
    ap.add_argument("--prompt-tokens", type=int, default=128)
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--judge-tp", type=int, default=0, help="0 = auto (largest valid TP <= ranks), 1 = GPU 0 only")
    ap.add_argument("--steps-per-graph", type=int, default=8)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--results-dir", default=os.path.join(ROOT, "bench", "results"),
                    help="rank 0 also writes the full record (per-step stats, p50/p90) here ('' = off)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    n_gpus = world
    # rehearsal mode for the multi-rank flow on a 1-GPU box: every rank on cuda:0, gloo collectives
    # (LLMC_BENCH_BACKEND=gloo LLMC_BENCH_SAME_GPU=1); the driver's runs use RCCL, one GPU per rank
    backend = os.environ.get("LLMC_BENCH_BACKEND", "nccl")
    gpu = 0 if os.environ.get("LLMC_BENCH_SAME_GPU") == "1" else local
    torch.cuda.set_device(gpu)
    dev = f"cuda:{gpu}"
    cdev = dev if backend == "nccl" else "cpu"  # where collective buffers live
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(dev))
        else:
            dist.init_process_group(backend)

    from llm_consensus_amd.consensus import build_judge_prompt, prompt_header
    from llm_consensus_amd.engine import Engine, EngineConfig, SamplingParams
    from llm_consensus_amd.models.config import FAMILIES
    from llm_consensus_amd.provider.base import Response
    from llm_consensus_amd.utils.tokenizer import get_tokenizer

    rcfg = FAMILIES[args.model]
    jcfg = FAMILIES[args.judge]
    mpg = args.models_per_gpu
    n_models = n_gpus * mpg
    jmax = args.judge_max_tokens or args.max_tokens
    tok = get_tokenizer(rcfg.vocab)
    jtok = get_tokenizer(jcfg.vocab)

    # synthetic prompt: seeded piece ids -> text (identical on every rank)
    g = torch.Generator().manual_seed(1234)
    pids = torch.randint(256, 256 + 60000, (args.prompt_tokens,), generator=g).tolist()
    prompt_text = tok.decode(pids).strip()
    prompt_ids = tok.encode(prompt_text, add_bos=True)

    resp_ctx = len(prompt_ids) + args.max_tokens + 64
    t0 = time.time()
    responders = []
    for j in range(mpg):
        idx = rank * mpg + j
        e = Engine(rcfg, EngineConfig(device=dev, max_context=resp_ctx, seed=1000 + idx,
                                      steps_per_graph=args.steps_per_graph, use_graphs=not args.no_graphs),
                   name=f"{args.model}@{idx}")
        responders.append((idx, e))
    judge = None
    judge_ctx = 0
    jtp = judge_tp_degree(jcfg, world, args.judge_tp) if n_models > 1 else 1
    from llm_consensus_amd.parallel.comm import TPGroup

    tp = TPGroup.single()
    if jtp > 1:
        # judge TP group = ranks 0..jtp-1 (the whole world by default); new_group is collective
        grp = dist.group.WORLD if jtp == world else dist.new_group(list(range(jtp)))
        ok = 1
        if rank < jtp:
            tp = TPGroup(grp, rank, jtp)
            # collective: every judge rank agrees on the outcome (peer mapping + a self-test)
            if not tp.enable_custom(dev):
                log("custom all-reduce unavailable; judge falls back to TP=1 on GPU 0")
                ok = 0
        flag = torch.tensor([ok], dtype=torch.int32, device=cdev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            jtp, tp = 1, TPGroup.single()
    if n_models > 1 and rank < jtp:
        # responses are decoded to text and re-tokenized by the judge: random byte tokens can expand
        # (invalid UTF-8 -> U+FFFD -> 3 byte tokens), so budget 2x per response
        judge_ctx = len(prompt_ids) + 1024 + n_models * (2 * args.max_tokens + 64) + jmax + 64
        judge = Engine(jcfg, EngineConfig(device=dev, max_context=judge_ctx, seed=777,
                                          steps_per_graph=args.steps_per_graph, use_graphs=not args.no_graphs),
                       tp=tp, name=f"{args.judge}@judge")
    # capture every decode graph up front (a capture beside another engine's running stream is
    # invalid; the worker process does the same before serving)
    if not args.no_graphs:
        for _, e in responders:
            e.warmup_graphs()
        if judge is not None:
            judge.warmup_graphs()
    torch.cuda.synchronize()
    log(f"engines ready in {time.time() - t0:.1f}s (responders {mpg}/gpu, judge ctx {judge_ctx})")

    def one_round(step: int):
        stats = {}
        t_start = time.perf_counter()
        # judge header prefill can start before any response exists
        jseq = None
        if judge is not None:
            jseq = judge.new_sequence()
            judge.prefill([jseq], [jtok.encode(prompt_header(prompt_text), add_bos=True)], want_logits=False)
        # co-located responders decode concurrently, one engine thread + hipStream each (as the
        # CLI's worker runs them)
        outs = [None] * len(responders)

        def run_one(j):
            idx, e = responders[j]
            outs[j] = e.generate_ids(prompt_ids, args.max_tokens, temperature=args.temperature,
                                     seed=1000 * step + idx + 1, stop_on_eos=False)

        if len(responders) == 1:
            run_one(0)
        else:
            ths = [threading.Thread(target=run_one, args=(j,)) for j in range(len(responders))]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
        t_resp = time.perf_counter()
        if rank == 0:
            log(f"round {step}: responders done in {t_resp - t_start:.2f}s")
        # gather responses to rank 0 (fixed-size int32 rows; RCCL over xGMI)
        local_t = torch.full((mpg, args.max_tokens), -1, dtype=torch.int32, device=dev)
        for j, ids in enumerate(outs):
            local_t[j, : len(ids)] = torch.tensor(ids, dtype=torch.int32, device=dev)
        if world > 1:
            all_t = torch.empty((world, mpg, args.max_tokens), dtype=torch.int32, device=cdev)
            dist.all_gather_into_tensor(all_t.view(world * mpg, args.max_tokens), local_t.to(cdev))
        else:
            all_t = local_t.unsqueeze(0)
        n_tokens = n_models * args.max_tokens
        if judge is not None:
            # every judge rank renders the same prompt from the gathered rows (deterministic), so
            # the TP shards prefill/decode in lockstep; rank 0 accounts the tokens
            rows = all_t.view(n_models, args.max_tokens).cpu().tolist()
            responses = []
            for i, r in enumerate(rows):
                r = [t for t in r if t >= 0]
                responses.append(Response(model=f"{args.model}@{i}", content=tok.decode(r), provider="rocm"))
            full = build_judge_prompt(prompt_text, responses)
            head = prompt_header(prompt_text)
            rest_ids = jtok.encode(full[len(head):])
            judge.prefill([jseq], [rest_ids])
            t_jp = time.perf_counter()
            if rank == 0:
                log(f"round {step}: judge prefill of {len(rest_ids)} tokens in {t_jp - t_resp:.2f}s (TP={jtp})")
            jids = judge.decode([jseq], [SamplingParams(jmax, args.temperature, 1.0, 0, 99 + step, False)])[0]
            stats["judge_prompt_tokens"] = jseq.length - len(jids)
            stats["judge_prefill_s"] = t_jp - t_resp
            stats["judge_decode_s"] = time.perf_counter() - t_jp
            if rank == 0:
                n_tokens += len(jids)
            judge.free_sequence(jseq)
            if judge.tp.custom is not None and judge.tp.custom.timed_out():
                log("WARNING: a custom all-reduce spin timed out (a peer stalled); judge tokens are suspect")
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t_end = time.perf_counter()
        stats["responders_s"] = t_resp - t_start
        stats["e2e_s"] = t_end - t_start
        stats["tokens"] = n_tokens
        return stats

    for w in range(args.warmup):
        st = one_round(w)
        log(f"warmup {w}: {st}")

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    lat = []
    tot_tokens = 0
    t0 = time.perf_counter()
    per_step = []
    for s in range(args.steps):
        st = one_round(100 + s)
        lat.append(st["e2e_s"])
        tot_tokens += st["tokens"]
        per_step.append(st)
        log(f"step {s}: {st}")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if rank == 0:
        value = tot_tokens / elapsed
        resp_tok_s = n_models * args.max_tokens * args.steps / sum(p["responders_s"] for p in per_step)
        out = {
            "metric": "consensus_aggregate_output_tokens_per_s",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed / args.steps, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic prompt (synthetic tokenizer), random-init weights",
            "config": {
                "model": f"{n_models}x {args.model} responders ({mpg}/GPU) + {args.judge} judge "
                         + (f"TP={jtp} on GPUs 0-{jtp - 1} (own streams)" if jtp > 1 else "on GPU0 stream"),
                "global_batch": n_models,
                "seq_len": len(prompt_ids) + args.max_tokens,
                "max_tokens": args.max_tokens,
                "prompt_tokens": len(prompt_ids),
                "parallelism": f"fanout{n_models}" + ("" if n_gpus == 1 else f"-dp{n_gpus}")
                               + (f"-judge_tp{jtp}" if jtp > 1 else ""),
            },
            "extra": {
                "p50_e2e_latency_s": round(statistics.median(lat), 3),
                "responder_decode_tok_s_per_model": round(resp_tok_s / n_models, 2),
                "judge_prompt_tokens": per_step[-1].get("judge_prompt_tokens", 0),
                "judge_prefill_s": round(per_step[-1].get("judge_prefill_s", 0.0), 3),
                "judge_decode_s": round(per_step[-1].get("judge_decode_s", 0.0), 3),
                "judge_tp": jtp,
            },
        }
        print(json.dumps(out), flush=True)
        if args.results_dir:
            srt = sorted(lat)
            rec = dict(out, per_step=per_step, p90_e2e_latency_s=round(srt[min(len(srt) - 1, int(0.9 * len(srt)))], 3),
                       time_utc=time.strftime("%Y%m%dT%H%M%SZ", time.gmtime()), argv=sys.argv[1:])
            try:
                os.makedirs(args.results_dir, exist_ok=True)
                fn = os.path.join(args.results_dir, f"bench_{rec['time_utc']}_n{n_gpus}.json")
                with open(fn, "w") as f:
                    json.dump(rec, f, indent=2)
            except OSError as e:
                log(f"could not write results record: {e}")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
