#!/usr/bin/env python3
"""Consensus-round benchmark (BASELINE.json metric: p50 end-to-end consensus latency + aggregate
output tokens/sec, N-model fan-out) for the BASELINE.json configs on N GPUs of one node.

One process per GPU (RCCL over xGMI). Under ``torchrun`` the ranks come from the environment;
``python bench.py --gpus N`` without a launcher starts its own N rank processes (GPU i = rank i)
before anything touches the GPU, and rank 0 prints the one JSON line. One timed step = one full
consensus round as ``llm-consensus`` runs it (reference ``internal/runner/runner.go:62-115``
fan-out, then ``internal/consensus/judge.go:81-104`` judge): every responder prefills the prompt
and decodes ``--max-tokens`` tokens, the responses are gathered, the judge prompt is rendered with
the reference template and the judge prefills it (header first, incrementally)
and decodes ``--max-tokens`` tokens.

``--config`` presets (the engines named in the JSON ``config.model`` are exactly the ones that run;
``config.name`` says which BASELINE config it is and, for a variant, how it differs):

* ``fanout`` (default; configs 2/3): ``max(3, N)`` Llama-3-8B responders (distinct random-init
  replicas ``llama-3-8b@i``) placed round-robin over the N GPUs, plus a Llama-3-8B judge
  tensor-parallel over the GPUs (``--judge-tp``, auto = largest valid degree <= N) on its own
  hipStreams beside the responders. N=1: 3 co-located responders + judge (config 2 on one GPU);
  N=4: 4 responders + TP=4 judge (variant of config 2); N=8: 8 responders + TP=8 judge (variant
  of config 3). ``--judge-tp 1`` puts the judge on the least-loaded GPU instead:
  ``--gpus 4 --n-models 3 --judge-tp 1`` is config 2 and ``--gpus 8 --judge-tp 1`` config 3 as
  BASELINE.json words them.
* ``--shared-weights`` (fanout, secondary preset, never the default): the replicas placed whole on
  one GPU share ONE weight copy and decode as rows of one batching engine (each with its own
  sampling seed) — BASELINE config 2's "replicas" taken literally; ``config.name`` says so.
* ``4``: 2 x Llama-3-70B responders, each TP=N/2 over its half of the node (RCCL + custom xGMI
  all-reduce), + Llama-3-8B judge. Needs an even N >= 2.
* ``5``: mixed fleet — Mixtral-8x7B (MoE grouped GEMM) + Llama-3-8B + Phi-3-mini responders, one
  per GPU, + Llama-3-70B judge TP=4 (long-context prefill). Needs N >= 4.

A config that does not fit N prints ONE JSON line with ``"skipped"`` and ``value`` null — never a
smaller config under the same name.

Round size: ``--max-tokens`` defaults to 2048 so that the driver's fixed ``--steps 20 --warmup 5``
finishes inside its 600-s limit at every N (N=1 measured: see BASELINE.md §2.0); 4096-token rounds
are the ``--max-tokens 4096`` secondary. Warmup rounds decode ``--warmup-tokens`` (default 64)
tokens per engine: every decode graph is captured when the engines are built and the judge's
prefill path is warmed once at full prompt length, so a short round exercises everything a timed
round does. The K timed rounds are always full rounds.

``--shapes tiny`` swaps every family for its tiny twin (same code paths; CPU / same-GPU
rehearsals of the multi-rank flows: ``LLMC_BENCH_DEVICE=cpu`` or ``LLMC_BENCH_SAME_GPU=1`` with
``LLMC_BENCH_BACKEND=gloo``).

Reported ``value`` = total generated tokens (responders + judge) per second of wall time over the
whole job (max over ranks); ``ms_per_step`` = mean round latency; p50/p90 are in ``extra``.
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
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
T_START = time.time()  # the wall-clock budget (--time-budget) counts from here

METRIC = "consensus_aggregate_output_tokens_per_s"
TINY = {"llama-3-8b": "llama-tiny", "llama-3-70b": "llama-tiny-tp4", "mixtral-8x7b": "mixtral-tiny",
        "phi-3-mini": "phi3-tiny"}


def log(*a):
    print(f"[bench r{os.environ.get('RANK', '0')}]", *a, file=sys.stderr, flush=True)


def self_launch(n: int) -> int:
    """Run this script as N rank processes (RANK = LOCAL_RANK = i binds GPU i; rendezvous on
    127.0.0.1) and return the first failing exit status, else 0. Called before anything imports
    torch, so the parent never initialises HIP; a rank that fails takes the others down (they
    would wait forever in a collective), and SIGTERM/SIGINT are forwarded."""
    import signal
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()

    signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    signal.signal(signal.SIGINT, lambda *a: (stop(), sys.exit(130)))
    status, kill_at = 0, None
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad and not status:
            status = bad[0]
            log(f"a rank exited with status {status}: stopping the others")
            stop()
            kill_at = time.time() + 15
        if kill_at is not None and time.time() > kill_at:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(0.2)
    if not status:
        status = next((p.returncode for p in procs if p.returncode), 0)
    return status


class Progress:
    """on_tokens callback that logs a token count every ``every`` seconds (rank 0): long phases
    (a judge decode on ranks time-sharing one GPU) keep writing instead of looking hung."""

    def __init__(self, what: str, every: float = 30.0):
        self.what, self.every, self.n = what, every, 0
        self.t0 = self.last = time.perf_counter()

    def __call__(self, *args) -> None:
        self.n += len(args[-1])
        now = time.perf_counter()
        if now - self.last >= self.every:
            self.last = now
            log(f"{self.what}: {self.n} tokens after {now - self.t0:.0f}s")


def judge_tp_degree(cfg, world: int, requested: int) -> int:
    """TP degree of the judge: ``requested`` if > 0, else the largest t <= min(world, 8) that
    shards the judge's heads, kv heads, FFN and vocab evenly (8 = custom all-reduce limit)."""
    if requested > 0:
        return requested
    for t in range(min(world, 8), 0, -1):
        if not (cfg.n_heads % t or cfg.n_kv_heads % t or cfg.intermediate % t or cfg.vocab % t):
            return t
    return 1


def make_plan(args, world: int):
    """(responders, judge, skip_reason): responders = [{name, family, ranks}], judge likewise.
    Ranks of a TP engine are consecutive global ranks; rank ranks[0] leads it."""
    fam = (lambda f: TINY.get(f, f)) if args.shapes == "tiny" else (lambda f: f)
    from llm_consensus_amd.models.config import FAMILIES

    if args.config == "fanout":
        n = args.n_models or max(3, world)
        rf = fam(args.model)
        # whole models round-robin over the GPUs; when n is not a multiple of N the remainder would
        # pile onto the first GPUs (N=2: GPU 0 decoding two models, GPU 1 one, the round waiting
        # on GPU 0), so each leftover responder is tensor-parallel over an equal share of the GPUs
        # instead: every GPU then streams the same bytes per step
        rt = args.resp_tp if world > 1 else 1
        if rt > 1 and world % rt == 0 and (n * rt) % world == 0 and judge_tp_degree(FAMILIES[rf], rt, 0) == rt:
            # --resp-tp t: every responder tensor-parallel over t consecutive GPUs, the groups
            # cycling over the N / t GPU groups, so each GPU hosts n t / N shards at once (N=8, t=2:
            # two half-models per GPU instead of one whole model)
            ng = world // rt
            resp = [{"name": f"{args.model}@{i}", "family": rf, "ranks": list(range((i % ng) * rt, (i % ng + 1) * rt)),
                     "seed": 1000 + i} for i in range(n)]
        else:
            whole = n - n % world if world > 1 else n
            rest = n - whole
            tp = world // rest if rest else 1
            if rest and (world % rest or judge_tp_degree(FAMILIES[rf], tp, 0) != tp):
                whole, rest = n, 0  # no even sharding: round-robin all of them
            resp = [{"name": f"{args.model}@{i}", "family": rf, "ranks": [i % world], "seed": 1000 + i}
                    for i in range(whole)]
            resp += [{"name": f"{args.model}@{whole + j}", "family": rf, "ranks": list(range(j * tp, (j + 1) * tp)),
                      "seed": 1000 + whole + j} for j in range(rest)]
        jf = fam(args.judge)
        jtp = judge_tp_degree(FAMILIES[jf], world, args.judge_tp)
        if jtp == 1:
            # a single-GPU judge time-shares the least-loaded GPU (config 2: the 4th GPU beside 3
            # responders; config 3: GPU 0 with one responder per GPU)
            load = [sum(g in e["ranks"] for e in resp) for g in range(world)]
            jranks = [min(range(world), key=lambda g: (load[g], g))]
        else:
            jranks = list(range(jtp))
        judge = {"name": f"{args.judge}@judge", "family": jf, "ranks": jranks, "seed": 777}
        return resp, judge, None
    if args.config == "4":
        if world < 2 or world % 2:
            return None, None, f"config 4 (2 x llama-3-70b TP=N/2 + llama-3-8b judge) needs an even N >= 2, got {world}"
        half = world // 2
        rf = fam("llama-3-70b")
        resp = [{"name": f"llama-3-70b@{i}", "family": rf, "ranks": list(range(i * half, (i + 1) * half)),
                 "seed": 1000 + i} for i in range(2)]
        jf = fam("llama-3-8b")
        jtp = judge_tp_degree(FAMILIES[jf], world, args.judge_tp)
        return resp, {"name": "llama-3-8b@judge", "family": jf, "ranks": list(range(jtp)), "seed": 777}, None
    if args.config == "5":
        if world < 4:
            return None, None, f"config 5 (mixed fleet + llama-3-70b TP=4 judge) needs N >= 4, got {world}"
        fleet = ["mixtral-8x7b", "llama-3-8b", "phi-3-mini"]
        resp = [{"name": f"{m}@0", "family": fam(m), "ranks": [i % world], "seed": 1000 + i} for i, m in enumerate(fleet)]
        jtp = args.judge_tp or 4
        # the 70B judge shards over the last 4 GPUs (off the responders' GPUs when N >= 7)
        return resp, {"name": "llama-3-70b@judge", "family": fam("llama-3-70b"),
                      "ranks": list(range(world - jtp, world)), "seed": 777}, None
    raise SystemExit(f"unknown --config {args.config}")


def colocated_tp(resp_plan, idx) -> bool:
    """Whether the tensor-parallel responder engine of plan entries ``idx`` shares a GPU with other
    responders that decode at the same time: it then keeps the separate (64-block) all-reduce
    launch instead of the row-parallel GEMVs' fused epilogue — the product path's rule
    (placement.fused_ar_allowed, used by LocalBackend for every worker)."""
    from llm_consensus_amd.parallel.placement import fused_ar_allowed

    gpus = {str(j): list(e["ranks"]) for j, e in enumerate(resp_plan)}
    return not fused_ar_allowed(gpus, str(idx[0]), [str(j) for j in range(len(resp_plan)) if j not in idx])


def responder_alone(resp_plan, idx) -> bool:
    """Whether the responder engine of plan entries ``idx`` decodes with no other responder on its
    GPUs (placement.decodes_alone, the product path's alone_plan): it then takes the lone-engine
    launch forms (ops.attn_oproj_min_chunk). The judge decodes after the responders: always alone."""
    from llm_consensus_amd.parallel.placement import decodes_alone

    if os.environ.get("LLMC_BENCH_SAME_GPU") == "1":
        # rehearsal: every rank's engine is on cuda:0, so no responder has its GPU to itself (the
        # fused attention + o_proj launch's waiting blocks would hold CUs the others need)
        return False
    gpus = {str(j): list(e["ranks"]) for j, e in enumerate(resp_plan)}
    return decodes_alone(gpus, str(idx[0]), [str(j) for j in range(len(resp_plan)) if j not in idx])


def config_name(args, world: int, resp, judge) -> str:
    """Which BASELINE.json config this run is, and how a variant differs from its wording."""
    if args.config != "fanout":
        return f"BASELINE config {args.config}"
    n, jtp = len(resp), len(judge["ranks"])
    whole = all(len(e["ranks"]) == 1 for e in resp)
    if world == 4 and n == 3 and jtp == 1 and whole:
        return "BASELINE config 2"
    if world == 8 and n == 8 and jtp == 1 and judge["ranks"] == [0] and whole:
        return "BASELINE config 3"
    if world == 1:
        return "BASELINE config 2 on one GPU (3 responders + judge co-located on their own streams)"
    base = "config 3" if world == 8 else "config 2"
    how = [f"{n} responders" + ("" if whole else " (some tensor-parallel)")]
    how.append(f"judge TP={jtp} over GPUs {judge['ranks'][0]}-{judge['ranks'][-1]}" if jtp > 1
               else f"judge on GPU {judge['ranks'][0]}")
    return f"variant of BASELINE {base} on {world} GPUs: " + ", ".join(how)


def describe(resp, judge) -> str:
    def one(e):
        tp = len(e["ranks"])
        return e["family"] + (f" TP={tp}" if tp > 1 else "")

    counts: Dict[str, int] = {}
    for e in resp:
        counts[one(e)] = counts.get(one(e), 0) + 1
    rs = " + ".join(f"{n}x {k}" for k, n in counts.items())
    j = one(judge)
    jr = judge["ranks"]
    where = f"GPU {jr[0]}" if len(jr) == 1 else f"GPUs {jr[0]}-{jr[-1]}"
    return f"{rs} responders + {j} judge on {where} (own streams)"


def topology(world: int, rank: int, dev: str, on_cpu: bool, tp_members, cdev) -> dict:
    """Collective (every rank): the node as this run saw it, for the JSON record.

    * ``dist_world_size``: the process group's size (``n_gpus`` only echoes WORLD_SIZE);
    * ``rank_devices``: per rank, its current device index and PCI bus id (CPU ranks: -1 / None);
    * ``peer_access``: rank 0's ``hipDeviceCanAccessPeer`` matrix over the visible devices (the
      gate the custom xGMI all-reduce's IPC mapping depends on);
    * ``allreduce_16k``: per TP engine group, the mean latency of a 16 KiB bf16 all-reduce over
      ``n`` back-to-back calls (custom one-shot kernel replayed from a HIP graph, else the group's
      torch.distributed backend eagerly), max over the group's ranks, measured before the warmups."""
    import socket

    import torch
    import torch.distributed as dist

    if on_cpu:
        mine = {"rank": rank, "device": -1, "pci_bus_id": None, "host": socket.gethostname()}
    else:
        idx = torch.cuda.current_device()
        props = torch.cuda.get_device_properties(idx)
        bus = None
        if hasattr(props, "pci_bus_id"):
            bus = f"{getattr(props, 'pci_domain_id', 0):04x}:{props.pci_bus_id:02x}:{getattr(props, 'pci_device_id', 0):02x}"
        mine = {"rank": rank, "device": idx, "pci_bus_id": bus, "host": socket.gethostname()}
    if world > 1:
        ranks_info = [None] * world
        dist.all_gather_object(ranks_info, mine)
    else:
        ranks_info = [mine]
    peer = []
    if not on_cpu and rank == 0:
        from llm_consensus_amd.utils.native import kernels

        n = torch.cuda.device_count()
        peer = [[int(kernels().can_access_peer(i, j)) for j in range(n)] for i in range(n)]
    lat = torch.zeros(max(1, len(tp_members)), dtype=torch.float64, device=cdev)
    impl = {}
    for gi, (name, ranks, tp) in enumerate(tp_members):
        if tp is None:
            continue
        n_calls = 1000 if not on_cpu else 50
        x = torch.ones(8192, dtype=torch.bfloat16, device=dev)
        if tp.custom is not None:
            impl[name] = "custom_oneshot"
            s = torch.cuda.Stream(torch.device(dev))
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                tp.custom.all_reduce_(x)  # eager once: kernel attributes, a live epoch
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(50):
                        tp.custom.all_reduce_(x)
                torch.cuda.synchronize()
                tp.barrier()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                for _ in range(n_calls // 50):
                    g.replay()
                b.record(s)
                torch.cuda.synchronize()
            us = 1000.0 * a.elapsed_time(b) / n_calls
            del g
        else:
            impl[name] = dist.get_backend(tp.group) if tp.group is not None else "none"
            tp.all_reduce_(x)
            if not on_cpu:
                torch.cuda.synchronize()
            tp.barrier()
            t = time.perf_counter()
            for _ in range(n_calls):
                tp.all_reduce_(x)
            if not on_cpu:
                torch.cuda.synchronize()
            us = 1e6 * (time.perf_counter() - t) / n_calls
        lat[gi] = us
    if world > 1:
        dist.all_reduce(lat, op=dist.ReduceOp.MAX)
        impls = [None] * world
        dist.all_gather_object(impls, impl)
        for d in impls:
            impl.update(d)
    return {
        "dist_world_size": dist.get_world_size() if world > 1 else 1,
        "rank_devices": ranks_info,
        "peer_access": peer,
        "allreduce_16k": {name: {"impl": impl.get(name), "ranks": ranks, "us": round(float(lat[gi]), 2)}
                          for gi, (name, ranks, _) in enumerate(tp_members)},
    }


def cli_path_bench(args) -> None:
    """The same consensus round through the shipping path (reference ``cmd/llm-consensus/main.go``
    132-170 + ``runner.go`` + ``judge.go``): ``ConsensusService`` places the engines once (worker
    processes, weights, graph capture: reported as ``startup_s``, outside the timed rounds), then
    every round is Runner fan-out -> LocalProvider -> worker pipe -> streamed detokenisation, the
    incrementally prefilled judge session, and the result persisted as ``data/<run-id>/``
    (result.json, prompt.txt, consensus.md) — with per-phase times."""
    import tempfile

    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        raise SystemExit("--path cli starts its own worker processes: run it without a launcher")
    if args.config != "fanout":
        raise SystemExit("--path cli: fanout preset only")
    from llm_consensus_amd.context import Context
    from llm_consensus_amd.output import encode_result
    from llm_consensus_amd.server import ConsensusService
    from llm_consensus_amd.utils.tokenizer import get_tokenizer
    from llm_consensus_amd.models.config import FAMILIES

    n = args.gpus
    fam = TINY.get(args.model, args.model) if args.shapes == "tiny" else args.model
    jfam = TINY.get(args.judge, args.judge) if args.shapes == "tiny" else args.judge
    n_resp = args.n_models or max(3, n)
    models = [f"{fam}@{i}" for i in range(n_resp)]
    judge = f"{jfam}@judge"
    jtp = judge_tp_degree(FAMILIES[jfam], n, args.judge_tp) if n > 1 else 0
    ptok = get_tokenizer(FAMILIES[fam].vocab)
    import random

    rng = random.Random(1234)
    prompt = ptok.decode([rng.randrange(256, min(256 + 60000, ptok.vocab_size - 2))
                          for _ in range(args.prompt_tokens)]).strip()
    t0 = time.perf_counter()
    svc = ConsensusService(models, judge, gpus=",".join(str(g) for g in range(n)), judge_tp=jtp if jtp > 1 else 0,
                           concurrency=1, timeout=3600.0, max_tokens=args.max_tokens, temperature=args.temperature)
    startup = time.perf_counter() - t0
    log(f"product path ready in {startup:.1f}s: {models} + {judge}")
    tmp = tempfile.mkdtemp(prefix="llmc-bench-cli-")

    def one_round(step: int, max_tokens: int):
        ev = []
        req = svc.parse({"prompt": prompt, "models": models, "judge": judge, "max_tokens": max_tokens,
                         "temperature": args.temperature, "seed": 1000 * step + 1})
        req["stop_on_eos"] = False  # full-length responses, as the engine-path bench decodes
        ts = time.perf_counter()
        res = svc.run(Context.background(), req, lambda name, data: ev.append((time.perf_counter() - ts, name, data)))
        t_run = time.perf_counter() - ts
        # persistence exactly as the CLI's auto-save (main.go:186-236)
        run_dir = os.path.join(tmp, f"run{step}")
        os.makedirs(run_dir, exist_ok=True)
        with open(os.path.join(run_dir, "prompt.txt"), "w") as f:
            f.write(prompt)
        with open(os.path.join(run_dir, "consensus.md"), "w") as f:
            f.write(res.consensus)
        with open(os.path.join(run_dir, "result.json"), "w") as f:
            f.write(encode_result(res))
        t_end = time.perf_counter() - ts
        done = [t for t, name, _ in ev if name == "model_done"]
        jstart = next((t for t, name, _ in ev if name == "judge_start"), t_run)
        jfirst = next((t for t, name, _ in ev if name == "judge_chunk"), t_run)
        jdone = next((d for _, name, d in ev if name == "judge_done"), {})
        resp_tokens = sum(r.output_tokens for r in res.responses)
        return {
            "e2e_s": t_end,
            "responders_s": max(done) if done else 0.0,
            "judge_start_s": jstart,
            "judge_ttft_s": jfirst - jstart,
            "judge_decode_s": t_run - jfirst,
            "persist_s": t_end - t_run,
            "tokens": resp_tokens + int(jdone.get("output_tokens", 0)),
            "response_tokens": [r.output_tokens for r in res.responses],
            "judge_tokens": int(jdone.get("output_tokens", 0)),
            "judge_prompt_tokens": int(jdone.get("prompt_tokens", 0)),
            "per_model_latency_ms": {r.model: r.latency_ms for r in res.responses},
            "per_model_ttft_ms": {r.model: round(r.ttft_ns / 1e6, 1) for r in res.responses},
        }

    try:
        for w in range(args.warmup):
            st = one_round(w, min(args.max_tokens, args.warmup_tokens or args.max_tokens))
            log(f"warmup {w}: {st}")
        per_step = []
        t0 = time.perf_counter()
        for s_ in range(args.steps):
            st = one_round(100 + s_, args.max_tokens)
            per_step.append(st)
            log(f"step {s_}: {st}")
        elapsed = time.perf_counter() - t0
    finally:
        svc.close()
    lat = [p["e2e_s"] for p in per_step]
    tot = sum(p["tokens"] for p in per_step)
    med = lambda k: round(statistics.median(p[k] for p in per_step), 3)  # noqa: E731
    out = {
        "metric": METRIC, "value": round(tot / elapsed, 2), "unit": "tokens/s", "n_gpus": n, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic prompt (synthetic tokenizer), random-init weights",
        "config": {"name": "product path (Runner -> LocalProvider -> worker -> pipe -> detokenizer -> result.json): "
                           + f"{n_resp} x {fam} + {jfam} judge on {n} GPU(s)",
                   "model": f"{n_resp}x {fam} responders + {jfam} judge" + (f" TP={jtp}" if jtp > 1 else ""),
                   "global_batch": n_resp, "seq_len": args.prompt_tokens + args.max_tokens,
                   "max_tokens": args.max_tokens, "prompt_tokens": args.prompt_tokens, "path": "cli",
                   "parallelism": f"fanout{n_resp}" + (f"-judge_tp{jtp}" if jtp > 1 else "")},
        "extra": {
            "startup_s": round(startup, 1),
            "p50_e2e_latency_s": round(statistics.median(lat), 3),
            "responders_s": med("responders_s"), "judge_start_s": med("judge_start_s"),
            "judge_ttft_s": med("judge_ttft_s"), "judge_decode_s": med("judge_decode_s"),
            "persist_s": med("persist_s"),
            "judge_prompt_tokens": per_step[-1]["judge_prompt_tokens"] if per_step else 0,
            "tokens_per_round": [p["tokens"] for p in per_step],
        },
    }
    print(json.dumps(out), flush=True)
    if args.results_dir:
        try:
            os.makedirs(args.results_dir, exist_ok=True)
            fn = os.path.join(args.results_dir, f"bench_cli_{time.strftime('%Y%m%dT%H%M%SZ', time.gmtime())}_n{n}.json")
            with open(fn, "w") as f:
                json.dump(dict(out, per_step=per_step, argv=sys.argv[1:]), f, indent=2)
        except OSError as e:
            log(f"could not write results record: {e}")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=0,
                    help="GPUs = ranks (default: WORLD_SIZE under a launcher, else 1); without a launcher, N > 1 "
                         "starts the N rank processes itself")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="fanout", choices=["fanout", "4", "5"])
    ap.add_argument("--shapes", default="full", choices=["full", "tiny"])
    ap.add_argument("--model", default="llama-3-8b", help="fanout: responder family")
    ap.add_argument("--judge", default="llama-3-8b", help="fanout: judge family")
    ap.add_argument("--n-models", type=int, default=0, help="fanout: responders (0 = max(3, N))")
    ap.add_argument("--max-tokens", type=int, default=2048,
                    help="tokens per response and for the judge (2048: 20 driver steps fit its 600-s limit)")
    ap.add_argument("--judge-max-tokens", type=int, default=0, help="0 = same as --max-tokens")
    ap.add_argument("--warmup-tokens", type=int, default=64,
                    help="tokens per engine in the (untimed) warmup rounds (0 = full rounds)")
    ap.add_argument("--prompt-tokens", type=int, default=128)
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--judge-tp", type=int, default=0, help="0 = auto (config 5: 4)")
    ap.add_argument("--resp-tp", type=int, default=1,
                    help="fanout, N > 1: every responder tensor-parallel over this many GPUs (1 = whole models "
                         "round-robin); ignored when it does not shard evenly")
    ap.add_argument("--shared-weights", action="store_true",
                    help="fanout secondary preset: the replicas placed whole on one GPU share ONE weight copy and "
                         "decode as rows of one engine (config.name says so; never the default)")
    ap.add_argument("--steps-per-graph", type=int, default=8)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--time-budget", type=float, default=560.0,
                    help="seconds the whole command may take (0 = off): the last two warmup rounds (W >= 2) are "
                         "timed at two lengths, and if K full rounds would overrun, the timed rounds decode fewer "
                         "tokens (recorded as config.max_tokens, with max_tokens_requested)")
    ap.add_argument("--path", default="engine", choices=["engine", "cli"],
                    help="engine: the engines driven directly on threads (the headline); cli: the product path "
                         "(Runner -> LocalProvider -> worker process -> pipe -> detokenizer -> result.json) through "
                         "ConsensusService with the same round, per-phase times in extra (fanout preset only)")
    ap.add_argument("--results-dir", default=os.path.join(ROOT, "bench", "results"),
                    help="rank 0 also writes the full record (per-step stats, p50/p90) here ('' = off)")
    args = ap.parse_args()

    if not args.gpus:
        args.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    if args.path == "cli":
        # the driver process of the product path never touches a GPU: its worker processes do
        return cli_path_bench(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start the N ranks here, before this process touches the GPU (it never
        # imports torch), and exit with their status
        sys.exit(self_launch(args.gpus))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}: one rank per GPU is the contract")
    n_gpus = world

    resp_plan, judge_plan, skip = make_plan(args, world)
    if skip is not None:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "tokens/s", "n_gpus": n_gpus,
                              "steps": args.steps, "warmup": args.warmup, "ms_per_step": None,
                              "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
                              "data": "synthetic", "skipped": skip,
                              "config": {"model": f"config {args.config}", "parallelism": "n/a"}}), flush=True)
        return

    # rehearsal modes for the multi-rank flow: every rank on cuda:0 (LLMC_BENCH_SAME_GPU=1) or on
    # the CPU (LLMC_BENCH_DEVICE=cpu), gloo collectives (LLMC_BENCH_BACKEND=gloo); the driver's
    # runs use RCCL, one GPU per rank
    on_cpu = os.environ.get("LLMC_BENCH_DEVICE") == "cpu"
    backend = "gloo" if on_cpu else os.environ.get("LLMC_BENCH_BACKEND", "nccl")
    if on_cpu:
        dev = "cpu"
    else:
        gpu = 0 if os.environ.get("LLMC_BENCH_SAME_GPU") == "1" else local
        torch.cuda.set_device(gpu)
        dev = f"cuda:{gpu}"
    cdev = dev if backend == "nccl" else "cpu"  # where collective buffers live

    def sync():
        if not on_cpu:
            torch.cuda.synchronize()

    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(dev))
        else:
            dist.init_process_group(backend)

    if os.environ.get("LLMC_BENCH_SAME_GPU") == "1":
        # ranks time-sharing one GPU without CU partitions: a peer's collective can wait well past
        # the 1-s spin bound meant for ranks that own their GPUs (car_proto.h kHostSpinTicks)
        os.environ.setdefault("LLMC_CAR_SPIN_S", "20")
        # ... and a TP replay of 8 decode steps over eight time-shared ranks takes ~6 s (round 4:
        # 11 ms per all-reduce): beyond the 5-s host deadline that fails a stalled replay
        os.environ.setdefault("LLMC_TP_STALL_S", "300")
        if os.environ.get("LLMC_BENCH_CU_SPLIT") == "1" and world > 1:
            # every rank's engines on a CU slice of their own, as on their own GPU: with eight ranks
            # time-sharing every CU, the spinning collectives of the ranks that have arrived hold the
            # CUs the last rank's kernels need (the custom all-reduce then times out)
            per = 256 // world
            os.environ.setdefault("LLMC_CU_MASK", f"{local * per}-{(local + 1) * per - 1}")
    from llm_consensus_amd import ops
    from llm_consensus_amd.consensus import build_judge_prompt, prompt_header
    from llm_consensus_amd.engine import Engine, EngineConfig, SamplingParams
    from llm_consensus_amd.models.config import FAMILIES
    from llm_consensus_amd.parallel.comm import TPGroup
    from llm_consensus_amd.provider.base import Response
    from llm_consensus_amd.utils.tokenizer import get_tokenizer

    jcfg = FAMILIES[judge_plan["family"]]
    jmax = args.judge_max_tokens or args.max_tokens
    jtok = get_tokenizer(jcfg.vocab)
    n_resp = len(resp_plan)

    # synthetic prompt: seeded piece ids -> text (identical on every rank)
    ptok = get_tokenizer(FAMILIES[resp_plan[0]["family"]].vocab)
    g = torch.Generator().manual_seed(1234)
    lo = 256
    pids = torch.randint(lo, min(lo + 60000, ptok.vocab_size - 2), (args.prompt_tokens,), generator=g).tolist()
    prompt_text = ptok.decode(pids).strip()

    tp_members = []  # (engine name, ranks, this rank's TPGroup or None) of every TP engine, plan order

    def tp_group(ranks: List[int]):
        """Collective over the world (dist.new_group): every rank calls it for every TP engine in
        plan order; returns this rank's TPGroup or None when it is not a member."""
        if len(ranks) == 1:
            return TPGroup.single() if rank == ranks[0] else None
        grp = dist.group.WORLD if len(ranks) == world else dist.new_group(ranks)
        if rank not in ranks:
            return None
        tp = TPGroup(grp, ranks.index(rank), len(ranks))
        if not on_cpu:
            # collective over the group: every member agrees on the outcome (peer mapping + a
            # self-test); on failure the group stays on RCCL (same-GPU rehearsals: gloo)
            tp.enable_custom(dev)
        return tp

    t0 = time.time()
    # responder engines: (plan indices, engine, prompt ids, tokenizer); one index per engine, or
    # with --shared-weights every replica placed whole on the same GPU as a row of one engine
    groups: List[List[int]] = []
    for i, e in enumerate(resp_plan):
        key = (e["family"], tuple(e["ranks"]))
        g = next((g for g in groups if args.shared_weights and len(e["ranks"]) == 1
                  and (resp_plan[g[0]]["family"], tuple(resp_plan[g[0]]["ranks"])) == key), None)
        if g is None:
            groups.append([i])
        else:
            g.append(i)
    responders = []
    for idx in groups:
        e = resp_plan[idx[0]]
        tp = tp_group(e["ranks"])
        if tp is None:
            if len(e["ranks"]) > 1:
                tp_members.append((e["name"] if len(idx) == 1 else "+".join(resp_plan[i]["name"] for i in idx),
                                   e["ranks"], None))
            continue
        cfg = FAMILIES[e["family"]]
        tok = get_tokenizer(cfg.vocab)
        ids = tok.encode(prompt_text, add_bos=True)
        ctx = len(ids) + args.max_tokens + 64
        graphs = not args.no_graphs and (tp.size == 1 or tp.custom is not None
                                         or (not on_cpu and tp.graph_capture_ok(dev)))
        name = e["name"] if len(idx) == 1 else "+".join(resp_plan[i]["name"] for i in idx)
        if tp.size > 1:
            tp_members.append((name, e["ranks"], tp))
        eng = Engine(cfg, EngineConfig(device=dev, max_context=ctx, seed=e["seed"], steps_per_graph=args.steps_per_graph,
                                       use_graphs=graphs, max_batch=len(idx),
                                       fused_ar=not colocated_tp(resp_plan, idx),
                                       attn_oproj_min_chunk=ops.attn_oproj_min_chunk(responder_alone(resp_plan, idx))),
                     tp=tp, name=name)
        responders.append((idx, eng, ids, tok))
    jtp_grp = tp_group(judge_plan["ranks"])
    if len(judge_plan["ranks"]) > 1:
        tp_members.append((judge_plan["name"], judge_plan["ranks"], jtp_grp))
    judge = None
    judge_ctx = 0
    if jtp_grp is not None:
        # responses are decoded to text and re-tokenized by the judge: random byte tokens can
        # expand (invalid UTF-8 -> U+FFFD -> 3 byte tokens), so budget 2x per response
        fixed = len(jtok.encode(build_judge_prompt(prompt_text, []), add_bos=True))
        judge_ctx = min(jcfg.max_position, fixed + n_resp * (2 * args.max_tokens + 64) + jmax + 64)
        graphs = not args.no_graphs and (jtp_grp.size == 1 or jtp_grp.custom is not None
                                         or (not on_cpu and jtp_grp.graph_capture_ok(dev)))
        judge = Engine(jcfg, EngineConfig(device=dev, max_context=judge_ctx, seed=judge_plan["seed"],
                                          steps_per_graph=args.steps_per_graph, use_graphs=graphs,
                                          attn_oproj_min_chunk=ops.attn_oproj_min_chunk(True)),
                       tp=jtp_grp, name=judge_plan["name"])
    # capture every decode graph up front (a capture beside another engine's running stream is
    # invalid; the worker process does the same before serving)
    for _, e, _, _ in responders:
        e.warmup_graphs()
    if judge is not None:
        judge.warmup_graphs()
        # the judge's prefill path at full prompt length once (allocator growth, every chunk
        # shape), so that short warmup rounds leave nothing for the first timed round to warm
        n_warm = min(judge_ctx - jmax - 64, fixed + n_resp * (args.max_tokens + 64))
        ws = judge.new_sequence()
        judge.prefill([ws], [[(7 * i) % 30000 + 300 for i in range(n_warm)]])
        judge.free_sequence(ws)
    sync()
    if world > 1:
        dist.barrier()
    log(f"engines ready in {time.time() - t0:.1f}s: {[e.name for _, e, _, _ in responders]}"
        + (f" + {judge.name} (TP={judge.tp.size}, ctx {judge_ctx})" if judge else ""))
    # what the run actually saw of the node (before any timed work): the RCCL world, each rank's
    # device, the peer-access matrix and every TP group's 16 KiB all-reduce latency
    topo = topology(world, rank, dev, on_cpu, tp_members, cdev)
    if rank == 0:
        log(f"topology: {topo}")

    def one_round(step: int, max_tokens: int = 0):
        max_tokens = max_tokens or args.max_tokens
        jmax_r = jmax if max_tokens == args.max_tokens else min(jmax, max_tokens)
        stats = {}
        t_start = time.perf_counter()
        # judge header prefill can start before any response exists
        jseq = None
        if judge is not None:
            jseq = judge.new_sequence()
            judge.prefill([jseq], [jtok.encode(prompt_header(prompt_text), add_bos=True)], want_logits=False)
        # co-located responders decode concurrently, one engine thread + hipStream each (as the
        # CLI's worker runs them); TP engines run in lockstep on every rank of their group
        outs: Dict[int, List[int]] = {}
        errs = []

        # per responder: [time to first token, latency] in s from the round start (its leader's clock)
        times = torch.zeros((n_resp, 2), dtype=torch.float64)

        def run_one(j):
            try:
                idx, e, ids, _ = responders[j]
                prog = Progress(f"round {step}: responder {idx[0]}") if (rank == 0 and j == 0) else None

                def on_tokens(r, new, prog=prog):
                    i = idx[r]
                    if times[i, 0] == 0:
                        times[i, 0] = time.perf_counter() - t_start
                    if prog is not None and r == 0:
                        prog(new)

                if len(idx) == 1:
                    outs[idx[0]] = e.generate_ids(ids, max_tokens, temperature=args.temperature,
                                                  seed=1000 * step + idx[0] + 1, stop_on_eos=False,
                                                  on_tokens=lambda new: on_tokens(0, new))
                else:  # replicas of one weight copy: rows of one batch, each with its own sampling seed
                    res = e.generate_batch([list(ids) for _ in idx],
                                           [SamplingParams(max_tokens, args.temperature, 1.0, 0, 1000 * step + i + 1,
                                                           False) for i in idx], on_tokens=on_tokens)
                    for i, r in zip(idx, res):
                        outs[i] = r
                done = time.perf_counter() - t_start
                for i in idx:
                    times[i, 1] = done
            except BaseException as ex:  # noqa: BLE001
                errs.append(ex)

        ths = [threading.Thread(target=run_one, args=(j,)) for j in range(len(responders))]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if errs:
            raise errs[0]
        t_resp = time.perf_counter()
        if rank == 0:
            log(f"round {step}: responders done in {t_resp - t_start:.2f}s")
        # gather every response to every rank: the leader of each responder writes its row
        # (token + 1; 0 = empty) and one SUM all-reduce assembles the table
        table = torch.zeros((n_resp, max_tokens), dtype=torch.int32)
        for idx, e, _, _ in responders:
            for i in idx:
                if e.tp.is_leader:
                    r = torch.tensor(outs[i], dtype=torch.int32) + 1
                    table[i, : r.numel()] = r
                else:
                    times[i] = 0.0  # the leader's clock reports this responder
        if world > 1:
            tt = table.to(cdev)
            dist.all_reduce(tt)
            table = tt.cpu()
            ts = times.to(cdev)
            dist.all_reduce(ts)
            times = ts.cpu()
        stats["per_model"] = {e["name"]: {"ttft_s": float(times[i, 0]), "latency_s": float(times[i, 1])}
                              for i, e in enumerate(resp_plan)}
        n_tokens = n_resp * max_tokens
        if judge is not None:
            # every judge rank renders the same prompt from the gathered rows (deterministic), so
            # the TP shards prefill/decode in lockstep; rank 0 accounts the judge tokens
            responses = []
            for i, e in enumerate(resp_plan):
                r = [t - 1 for t in table[i].tolist() if t > 0]
                rtok = get_tokenizer(FAMILIES[e["family"]].vocab)
                responses.append(Response(model=e["name"], content=rtok.decode(r), provider="rocm"))
            # Why every response block is prefilled here, after the LAST response, while the product
            # path (provider/local.py) extends the judge session as EACH response
            # completes: (1) on N > 1 ranks the blocks must be identical and in the same order on
            # every judge rank, and the responses only meet on every rank through the collective
            # gather above; (2) the bench's responders all decode exactly max_tokens, so they
            # complete within milliseconds of each other and the product path also has every block
            # left to prefill once the last one lands. The product path itself is timed by
            # `--path cli` (within +0.5 % of this engine path).
            full = build_judge_prompt(prompt_text, responses)
            head = prompt_header(prompt_text)
            rest_ids = jtok.encode(full[len(head):])
            judge.prefill([jseq], [rest_ids])
            sync()
            t_jp = time.perf_counter()
            if rank == 0:
                log(f"round {step}: judge prefill of {len(rest_ids)} tokens in {t_jp - t_resp:.2f}s (TP={judge.tp.size})")
            jprog = Progress(f"round {step}: judge") if rank == 0 else None
            jfirst = []

            def on_judge_tokens(i, new):
                if not jfirst:
                    jfirst.append(time.perf_counter())
                if jprog is not None:
                    jprog(i, new)

            jids = judge.decode([jseq], [SamplingParams(jmax_r, args.temperature, 1.0, 0, 99 + step, False)],
                                on_tokens=on_judge_tokens)[0]
            stats["judge_ttft_s"] = (jfirst[0] if jfirst else time.perf_counter()) - t_resp
            stats["judge_prompt_tokens"] = jseq.length - len(jids)
            stats["judge_prefill_s"] = t_jp - t_resp
            stats["judge_decode_s"] = time.perf_counter() - t_jp
            if judge.tp.is_leader:
                stats["judge_tokens"] = len(jids)
            judge.free_sequence(jseq)
        sync()
        # a custom-collective spin that gave up means a peer stalled and the sums are invalid
        for e in [e for _, e, _, _ in responders] + ([judge] if judge is not None else []):
            if e.tp.size > 1 and e.tp.custom_timed_out():
                raise RuntimeError(f"{e.name}: a custom all-reduce spin timed out (a peer stalled): tokens are invalid")
        if world > 1:
            dist.barrier()
        t_end = time.perf_counter()
        stats["responders_s"] = t_resp - t_start
        stats["e2e_s"] = t_end - t_start
        stats["tokens"] = n_tokens + (jmax_r if judge_plan else 0)
        return stats

    wt = args.warmup_tokens or args.max_tokens
    probe = {}
    for w in range(args.warmup):
        # the last two warmup rounds double as a cost probe: round time ~ c0 + c1 x tokens
        n_w = 2 * wt if (w == args.warmup - 1 and args.warmup >= 2) else wt
        tw = time.perf_counter()
        st = one_round(w, min(n_w, args.max_tokens))
        probe[min(n_w, args.max_tokens)] = time.perf_counter() - tw
        log(f"warmup {w}: {st}")
    round_tokens = args.max_tokens
    if args.time_budget > 0 and args.warmup >= 2 and len(probe) == 2:
        (t1, s1), (t2, s2) = sorted(probe.items())
        pr = torch.tensor([s1, s2], dtype=torch.float64, device=cdev)
        if world > 1:
            dist.all_reduce(pr, op=dist.ReduceOp.MAX)
        s1, s2 = float(pr[0]), float(pr[1])
        c1 = max((s2 - s1) / (t2 - t1), 1e-6)
        c0 = max(s1 - c1 * t1, 0.0)
        left = args.time_budget - (time.time() - T_START) - 10.0  # teardown margin
        # x 1.15: the probe rounds are short, and a full round's attention and judge prompt grow
        # with its length (the two-point line under-estimates it)
        need = 1.15 * args.steps * (c0 + c1 * args.max_tokens)
        if need > left:
            fit = int(((left / (1.15 * args.steps)) - c0) / c1) // 64 * 64
            round_tokens = max(64, min(args.max_tokens, fit))
            log(f"time budget: {args.steps} rounds of {args.max_tokens} tokens need ~{need:.0f}s, {left:.0f}s left: "
                f"timed rounds decode {round_tokens} tokens")

    sync()
    # the custom collectives' wait statistics count the timed rounds only (a collective resync of
    # every TP engine this rank holds, in plan order)
    for e in [e for _, e, _, _ in responders] + ([judge] if judge is not None else []):
        if e.tp.size > 1:
            e.tp.resync_collectives()
    if world > 1:
        dist.barrier()
    lat = []
    tot_tokens = 0
    t0 = time.perf_counter()
    per_step = []
    for s in range(args.steps):
        st = one_round(100 + s, round_tokens)
        lat.append(st["e2e_s"])
        tot_tokens += st["tokens"]
        per_step.append(st)
        log(f"step {s}: {st}")
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    judge_stats = per_step[-1] if per_step else {}
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        # judge timings live on the judge's ranks: rank 0 is not one of them in config 5 at N > 4
        jt = torch.tensor([judge_stats.get(k, 0.0) for k in ("judge_prompt_tokens", "judge_prefill_s",
                                                             "judge_decode_s", "judge_ttft_s")],
                          dtype=torch.float64, device=cdev)
        dist.all_reduce(jt, op=dist.ReduceOp.MAX)
        judge_stats = dict(judge_stats, judge_prompt_tokens=int(jt[0].item()), judge_prefill_s=float(jt[1].item()),
                           judge_decode_s=float(jt[2].item()), judge_ttft_s=float(jt[3].item()))
    # every TP engine's custom-collective state at the end, from every rank that holds a shard
    ar_state = {e.name: {"custom": e.tp.custom is not None,
                         "fused": e.tp.custom_fused is not None and e.ecfg.fused_ar,
                         "timed_out": bool(e.tp.custom_timed_out()),
                         "max_wait_us": e.tp.collective_max_wait_us()}
                for e in [e for _, e, _, _ in responders] + ([judge] if judge is not None else []) if e.tp.size > 1}
    if world > 1:
        allst = [None] * world
        dist.all_gather_object(allst, ar_state)
        ar_state = {}
        for d in allst:
            for k, v in d.items():
                cur = ar_state.setdefault(k, {"custom": True, "fused": True, "timed_out": False, "max_wait_us": {}})
                cur["custom"] = cur["custom"] and v["custom"]
                cur["fused"] = cur["fused"] and v["fused"]
                cur["timed_out"] = cur["timed_out"] or v["timed_out"]
                for c, us in v["max_wait_us"].items():  # the longest wait of any rank
                    cur["max_wait_us"][c] = max(cur["max_wait_us"].get(c, 0.0), us)
    if rank == 0:
        names = [e["name"] for e in resp_plan]
        value = tot_tokens / elapsed
        resp_tok_s = n_resp * round_tokens * args.steps / sum(p["responders_s"] for p in per_step)
        jtp = len(judge_plan["ranks"])
        rtp = sorted({len(e["ranks"]) for e in resp_plan if len(e["ranks"]) > 1})
        par = {"fanout": f"fanout{n_resp}" + "".join(f"-resp_tp{t}" for t in rtp)
               + ("-shared_weights" if any(len(g) > 1 for g, _, _, _ in responders) else ""),
               "4": f"fanout2-tp{len(resp_plan[0]['ranks'])}", "5": "fanout3-mixed"}[args.config]
        shortened = round_tokens < args.max_tokens
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed / args.steps, 2),
            "higher_is_better": True,
            # fanout: responders grow with N (one per GPU from N=3); configs 4/5 fix the fleet
            "scaling": "weak" if args.config == "fanout" else "strong",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic prompt (synthetic tokenizer), random-init weights",
            "config": {
                "name": config_name(args, n_gpus, resp_plan, judge_plan)
                + (" [secondary preset: replicas on one GPU share one weight copy, batched as rows of one engine]"
                   if args.shared_weights else "")
                + (f" [budget-shortened: {round_tokens}-token rounds instead of {args.max_tokens}]" if shortened else ""),
                "model": describe(resp_plan, judge_plan),
                "global_batch": n_resp,
                "seq_len": args.prompt_tokens + round_tokens,
                "max_tokens": round_tokens,
                "prompt_tokens": args.prompt_tokens,
                "parallelism": par + ("" if n_gpus == 1 else f"-over{n_gpus}gpus") + (f"-judge_tp{jtp}" if jtp > 1 else ""),
            },
            "extra": {
                "p50_e2e_latency_s": round(statistics.median(lat), 3),
                "p90_e2e_latency_s": round(sorted(lat)[min(len(lat) - 1, int(0.9 * len(lat)))], 3),
                "responders_s": round(statistics.median(p["responders_s"] for p in per_step), 3),
                "responder_decode_tok_s_per_model": round(resp_tok_s / n_resp, 2),
                "judge_prompt_tokens": judge_stats.get("judge_prompt_tokens", 0),
                "judge_prefill_s": round(judge_stats.get("judge_prefill_s", 0.0), 3),
                "judge_decode_s": round(judge_stats.get("judge_decode_s", 0.0), 3),
                # the judge's first token after the last response (incremental prefill + one sample)
                "judge_ttft_s": round(judge_stats.get("judge_ttft_s", 0.0), 3),
                # per responder, median over the timed rounds (reference result.json latency_ms;
                # raw ns as the reference's time.Duration would hold it)
                "per_model_latency_ms": {m: round(1000 * statistics.median(p["per_model"][m]["latency_s"]
                                                                          for p in per_step), 1) for m in names},
                "per_model_latency_ns": {m: int(1e9 * statistics.median(p["per_model"][m]["latency_s"]
                                                                       for p in per_step)) for m in names},
                "per_model_ttft_ms": {m: round(1000 * statistics.median(p["per_model"][m]["ttft_s"] for p in per_step), 1)
                                      for m in names},
                "judge_tp": jtp,
                "warmup_rounds_tokens": [min(args.max_tokens, wt * (2 if (w == args.warmup - 1 and args.warmup >= 2)
                                                                      else 1)) for w in range(args.warmup)],
                "max_tokens_requested": args.max_tokens,
                "budget_shortened": shortened,
                "time_budget_s": args.time_budget,
                "custom_allreduce": {k: v["custom"] for k, v in ar_state.items()},
                "custom_allreduce_timed_out": {k: v["timed_out"] for k, v in ar_state.items()},
                # the row-parallel decode GEMVs' all-reduce fused into their epilogue (EPI_AR)
                "fused_rowparallel_allreduce": {k: v["fused"] for k, v in ar_state.items()},
                # per TP engine and collective buffer (oneshot / twoshot / fused), the longest time a
                # rank's spin waited on its peers during the timed rounds, us (device counter; the
                # spins give up at 1 s)
                "collective_max_wait_us": {k: v["max_wait_us"] for k, v in ar_state.items()},
                **topo,
            },
        }
        print(json.dumps(out), flush=True)
        if args.results_dir:
            rec = dict(out, per_step=per_step, time_utc=time.strftime("%Y%m%dT%H%M%SZ", time.gmtime()),
                       argv=sys.argv[1:])
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
