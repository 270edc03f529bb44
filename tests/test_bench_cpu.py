"""bench.py multi-rank flows on CPU ranks (gloo, oracle ops, tiny shapes): the fan-out with a TP
judge, config 4 (two TP=2 responder groups + judge) and config 5 (mixed Mixtral/Llama/Phi-3 fleet +
TP=4 judge), and the explicit "skipped" record of a config that does not fit the GPU count."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _run(n, args, port):
    env = dict(os.environ, LLMC_BENCH_DEVICE="cpu", OMP_NUM_THREADS="1")
    cmd = ([sys.executable, "bench.py"] if n == 1 else
           [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
            "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", str(n)])
    r = subprocess.run(cmd + args + ["--results-dir", ""], cwd=ROOT, capture_output=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1
    return json.loads(lines[0])


def _tokens_ok(d, max_tokens):
    tokens = (d["config"]["global_batch"] + 1) * max_tokens
    assert abs(d["value"] - tokens / (d["ms_per_step"] / 1000)) < 0.02 * d["value"]
    assert d["extra"]["judge_prompt_tokens"] > 0 and d["extra"]["judge_decode_s"] > 0
    # per-model latency / TTFT of every responder, whichever rank ran it
    lat, ttft = d["extra"]["per_model_latency_ms"], d["extra"]["per_model_ttft_ms"]
    assert len(lat) == d["config"]["global_batch"] and set(lat) == set(ttft)
    assert all(0 < ttft[m] <= lat[m] for m in lat)
    assert 0 < d["extra"]["judge_ttft_s"] < d["ms_per_step"] / 1000


def test_fanout_one_rank_runs_judge():
    d = _run(1, ["--shapes", "tiny", "--steps", "1", "--warmup", "0", "--max-tokens", "12"], 0)
    assert d["config"]["global_batch"] == 3 and d["scaling"] == "weak"
    _tokens_ok(d, 12)


def test_shared_weights_preset_batches_replicas_as_rows():
    """--shared-weights: the three replicas on the one GPU are rows of ONE engine (one weight copy),
    every responder still returns its own tokens and per-model timings; the config name and the
    parallelism label say it is the secondary preset."""
    d = _run(1, ["--shapes", "tiny", "--steps", "1", "--warmup", "1", "--max-tokens", "12", "--shared-weights"], 0)
    assert d["config"]["global_batch"] == 3
    assert "secondary preset" in d["config"]["name"] and d["config"]["parallelism"].endswith("-shared_weights")
    _tokens_ok(d, 12)
    lat = d["extra"]["per_model_latency_ms"]
    assert len(set(lat.values())) == 1  # one batch: every replica finishes with it


def test_config4_two_tp_groups():
    d = _run(4, ["--config", "4", "--shapes", "tiny", "--steps", "1", "--warmup", "0", "--max-tokens", "12"], 29691)
    assert d["config"]["name"] == "BASELINE config 4" and d["scaling"] == "strong"
    assert d["config"]["model"].startswith("2x llama-tiny-tp4 TP=2 responders")
    _tokens_ok(d, 12)


def test_config5_mixed_fleet_tp4_judge():
    d = _run(4, ["--config", "5", "--shapes", "tiny", "--steps", "1", "--warmup", "0", "--max-tokens", "12"], 29692)
    assert "mixtral-tiny" in d["config"]["model"] and "phi3-tiny" in d["config"]["model"]
    assert d["extra"]["judge_tp"] == 4
    _tokens_ok(d, 12)


def test_config_too_big_is_skipped_not_shrunk():
    for cfg in ("4", "5"):
        d = _run(1, ["--config", cfg, "--steps", "1", "--warmup", "0"], 0)
        assert d["value"] is None and "needs" in d["skipped"]


def test_fanout_eight_ranks_like_the_scale_run():
    """The driver's N=8 scaling run, rehearsed on 8 gloo ranks: one responder per rank, the judge
    tensor-parallel over the first ranks its head count allows, value = whole-job tokens/s."""
    d = _run(8, ["--shapes", "tiny", "--steps", "1", "--warmup", "0", "--max-tokens", "12"], 29693)
    assert d["n_gpus"] == 8 and d["config"]["global_batch"] == 8 and d["scaling"] == "weak"
    assert d["extra"]["judge_tp"] >= 2
    _tokens_ok(d, 12)


def test_fanout_responders_tensor_parallel_pairs():
    """--resp-tp 2 on 4 gloo ranks: four TP=2 responders, two per rank pair, and the TP=4 judge."""
    d = _run(4, ["--shapes", "tiny", "--steps", "1", "--warmup", "0", "--max-tokens", "12", "--resp-tp", "2"], 29695)
    assert d["config"]["global_batch"] == 4
    assert "4x llama-tiny TP=2 responders" in d["config"]["model"]
    _tokens_ok(d, 12)


def test_fanout_two_ranks_balances_the_third_responder():
    """N=2: two whole responders (one per rank) and the third tensor-parallel over both ranks, so
    both GPUs stream the same bytes per step; the judge is TP=2."""
    d = _run(2, ["--shapes", "tiny", "--steps", "1", "--warmup", "0", "--max-tokens", "12"], 29694)
    assert d["config"]["global_batch"] == 3
    assert "2x llama-tiny + 1x llama-tiny TP=2 responders" in d["config"]["model"]
    assert d["config"]["parallelism"] == "fanout3-resp_tp2-over2gpus-judge_tp2"
    _tokens_ok(d, 12)


def test_warmup_rounds_are_short_timed_rounds_full():
    """Warmup rounds decode --warmup-tokens per engine (the last one twice that: with the one
    before it, the round-cost probe of the time budget); the timed rounds (and the reported
    tokens) are full rounds."""
    d = _run(1, ["--shapes", "tiny", "--steps", "1", "--warmup", "3", "--max-tokens", "12", "--warmup-tokens", "4"], 0)
    assert d["extra"]["warmup_rounds_tokens"] == [4, 4, 8]
    assert d["config"]["max_tokens"] == d["extra"]["max_tokens_requested"] == 12
    _tokens_ok(d, 12)


def test_time_budget_shortens_rounds_never_steps():
    """A budget the requested rounds cannot fit: the timed rounds decode fewer tokens (reported as
    config.max_tokens next to max_tokens_requested), still exactly --steps of them."""
    d = _run(1, ["--shapes", "tiny", "--steps", "2", "--warmup", "2", "--max-tokens", "4096", "--warmup-tokens", "8",
                 "--time-budget", "1"], 0)
    assert d["steps"] == 2 and d["extra"]["max_tokens_requested"] == 4096
    assert 64 <= d["config"]["max_tokens"] < 4096
    assert d["extra"]["budget_shortened"] is True and "budget-shortened" in d["config"]["name"]
    _tokens_ok(d, d["config"]["max_tokens"])


def _self_launched(n, extra=()):
    """``python bench.py --gpus N`` with no launcher in the environment: bench.py starts the N
    rank processes itself."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(LLMC_BENCH_DEVICE="cpu", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--shapes", "tiny", "--steps", "1", "--warmup",
                        "1", "--max-tokens", "8", "--warmup-tokens", "4", "--results-dir", "", *extra],
                       cwd=ROOT, capture_output=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout.decode()
    return json.loads(lines[0])


def test_self_launch_n_ranks_without_a_launcher():
    """Self-launched N ranks, and the record proves what the job saw: the process-group size, one
    device entry per rank, every TP group's measured 16 KiB all-reduce latency and its
    custom-collective state (CPU ranks: device -1, gloo, no custom kernels)."""
    for n in (2, 4, 8):
        d = _self_launched(n)
        assert d["n_gpus"] == n and d["steps"] == 1 and d["warmup"] == 1
        assert d["config"]["global_batch"] == max(3, n)
        _tokens_ok(d, 8)
        x = d["extra"]
        assert x["dist_world_size"] == n and x["budget_shortened"] is False
        assert [r["rank"] for r in x["rank_devices"]] == list(range(n))
        assert all(r["device"] == -1 for r in x["rank_devices"]) and x["peer_access"] == []
        judge = [k for k in x["allreduce_16k"] if k.endswith("@judge")]
        assert judge and x["allreduce_16k"][judge[0]]["impl"] == "gloo"
        assert x["allreduce_16k"][judge[0]]["us"] > 0 and len(x["allreduce_16k"][judge[0]]["ranks"]) == x["judge_tp"]
        assert set(x["custom_allreduce"]) == set(x["custom_allreduce_timed_out"]) == set(x["allreduce_16k"])
        assert not any(x["custom_allreduce"].values()) and not any(x["custom_allreduce_timed_out"].values())
        # the longest peer wait per TP engine and collective buffer (none without custom kernels)
        assert set(x["collective_max_wait_us"]) == set(x["custom_allreduce"])
        assert all(v == {} for v in x["collective_max_wait_us"].values())


def test_gpus_defaults_to_world_size_under_a_launcher():
    """torchrun without --gpus: the rank count comes from WORLD_SIZE (an explicit mismatch fails)."""
    env = dict(os.environ, LLMC_BENCH_DEVICE="cpu", OMP_NUM_THREADS="1")
    base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
            "127.0.0.1", "--master-port", "29695", "bench.py", "--shapes", "tiny", "--steps", "1", "--warmup", "0",
            "--max-tokens", "8", "--results-dir", ""]
    r = subprocess.run(base, cwd=ROOT, capture_output=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    d = json.loads([ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")][0])
    assert d["n_gpus"] == 2 and d["extra"]["dist_world_size"] == 2
    base[base.index("29695")] = "29696"
    r = subprocess.run(base + ["--gpus", "4"], cwd=ROOT, capture_output=True, timeout=600, env=env)
    assert r.returncode != 0 and b"WORLD_SIZE" in r.stderr


def test_self_launch_failing_rank_fails_the_job():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(LLMC_BENCH_DEVICE="cpu", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--shapes", "tiny", "--model", "no-such-family",
                        "--steps", "1", "--warmup", "0", "--results-dir", ""],
                       cwd=ROOT, capture_output=True, timeout=300, env=env)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")]


def test_config_names_are_honest():
    """Config 2 / 3 as BASELINE.json words them with --judge-tp 1; the TP-judge defaults are
    labelled variants."""
    import argparse

    import bench

    def plan(n, **kw):
        a = argparse.Namespace(config="fanout", shapes="full", model="llama-3-8b", judge="llama-3-8b",
                               n_models=kw.get("n_models", 0), judge_tp=kw.get("judge_tp", 0),
                               resp_tp=kw.get("resp_tp", 1))
        r, j, _ = bench.make_plan(a, n)
        return bench.config_name(a, n, r, j), r, j

    name, r, j = plan(4, n_models=3, judge_tp=1)
    assert name == "BASELINE config 2" and j["ranks"] == [3] and [e["ranks"] for e in r] == [[0], [1], [2]]
    name, r, j = plan(8, judge_tp=1)
    assert name == "BASELINE config 3" and j["ranks"] == [0] and len(r) == 8
    name, _, j = plan(8)
    assert name.startswith("variant of BASELINE config 3") and "TP=8" in name and len(j["ranks"]) == 8
    name, _, _ = plan(4)
    assert name.startswith("variant of BASELINE config 2") and "4 responders" in name
    name, _, j = plan(1)
    assert name.startswith("BASELINE config 2 on one GPU") and j["ranks"] == [0]
    # --resp-tp 2 at N=8: 8 responders TP=2, two per GPU pair (every GPU hosts two half-models)
    name, r, _ = plan(8, resp_tp=2)
    assert [e["ranks"] for e in r] == [[0, 1], [2, 3], [4, 5], [6, 7]] * 2 and "some tensor-parallel" in name
    _, r, _ = plan(4, resp_tp=2)
    assert [e["ranks"] for e in r] == [[0, 1], [2, 3]] * 2
    _, r, _ = plan(1, resp_tp=2)  # one GPU: whole models whatever the flag
    assert [e["ranks"] for e in r] == [[0]] * 3
    # a TP responder sharing its GPUs with other responders keeps the separate all-reduce launch
    _, r, _ = plan(2)  # N=2: the third responder is TP=2 over both GPUs, beside the two whole ones
    assert [bench.colocated_tp(r, [i]) for i in range(3)] == [False, False, True]
    _, r, _ = plan(8, resp_tp=2)
    assert all(bench.colocated_tp(r, [i]) for i in range(8))
    _, r, _ = plan(8)
    assert not any(bench.colocated_tp(r, [i]) for i in range(8))


def test_product_path_round_reports_phases():
    """--path cli: the same round through ConsensusService (Runner -> LocalProvider -> worker
    process -> pipe -> detokenizer -> persisted result), full-length responses, per-phase times."""
    env = dict(os.environ, LLMC_DEVICE="cpu", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "bench.py", "--path", "cli", "--shapes", "tiny", "--steps", "1", "--warmup", "1",
                        "--max-tokens", "12", "--warmup-tokens", "4", "--results-dir", ""],
                       cwd=ROOT, capture_output=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    d = json.loads([ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")][0])
    assert d["config"]["path"] == "cli" and d["config"]["global_batch"] == 3
    x = d["extra"]
    assert x["tokens_per_round"] == [4 * 12]  # 3 full responses + the judge, EOS ignored as in the engine bench
    assert 0 < x["responders_s"] <= x["judge_start_s"] < d["ms_per_step"] / 1000
    assert x["judge_prompt_tokens"] > 0 and x["judge_decode_s"] > 0 and x["persist_s"] >= 0
