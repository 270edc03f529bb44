"""bench.py driver contract on the GPU box: one JSON line with the required keys, whole-job
value consistent with steps x tokens / time, for 1 rank (3 co-located responders + judge: a real
consensus round) and for same-GPU gloo rehearsals of the multi-rank flows (every rank on cuda:0):
the fan-out with a TP=2 judge, config 4 (two TP responder groups) and config 5 (mixed fleet +
TP=4 judge) at tiny shapes."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def check_line(line, n_gpus, steps, warmup, max_tokens, scaling="weak"):
    d = json.loads(line)
    assert KEYS <= set(d), set(d) ^ KEYS
    assert d["n_gpus"] == n_gpus and d["steps"] == steps and d["warmup"] == warmup
    assert d["higher_is_better"] is True and d["scaling"] == scaling and d["dtype"] == "bf16"
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(d["config"])
    tokens = (d["config"]["global_batch"] + 1) * max_tokens  # responders + judge
    assert abs(d["value"] - tokens * steps / (d["ms_per_step"] * steps / 1000)) < 0.02 * d["value"]
    assert d["extra"]["judge_prompt_tokens"] > 0 and d["extra"]["judge_decode_s"] > 0
    return d


def run_ranks(n, args, port, env_extra=None, timeout=600):
    env = dict(os.environ, **(env_extra or {}))
    if n == 1:
        cmd = [sys.executable, "bench.py"]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
               "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", str(n)]
    r = subprocess.run(cmd + args + ["--results-dir", ""], cwd=ROOT, capture_output=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1  # rank 0 only
    return lines[0]


def test_bench_json_contract_1gpu(cuda):
    line = run_ranks(1, ["--model", "llama-small", "--judge", "llama-small", "--steps", "2", "--warmup", "1",
                         "--max-tokens", "48"], 0)
    d = check_line(line, 1, 2, 1, 48)
    assert d["config"]["global_batch"] == 3  # N=1: three co-located responders + the judge


SAME_GPU = {"LLMC_BENCH_BACKEND": "gloo", "LLMC_BENCH_SAME_GPU": "1"}


def test_bench_two_rank_rehearsal(cuda):
    line = run_ranks(2, ["--model", "llama-small", "--judge", "llama-small", "--steps", "1", "--warmup", "1",
                         "--max-tokens", "32"], 29631, SAME_GPU)
    d = check_line(line, 2, 1, 1, 32)
    assert d["extra"]["judge_tp"] == 2


def test_bench_config4_rehearsal(cuda):
    line = run_ranks(4, ["--config", "4", "--shapes", "tiny", "--steps", "1", "--warmup", "0", "--max-tokens", "24"],
                     29632, SAME_GPU)
    d = check_line(line, 4, 1, 0, 24, scaling="strong")
    assert d["config"]["global_batch"] == 2 and "TP=2 responders" in d["config"]["model"]
    assert d["extra"]["custom_allreduce"]["llama-3-70b@0"] is True  # TP decode through the custom kernels


def test_bench_config5_rehearsal(cuda):
    line = run_ranks(4, ["--config", "5", "--shapes", "tiny", "--steps", "1", "--warmup", "0", "--max-tokens", "24"],
                     29633, SAME_GPU)
    d = check_line(line, 4, 1, 0, 24, scaling="strong")
    assert "mixtral-tiny" in d["config"]["model"] and d["extra"]["judge_tp"] == 4
