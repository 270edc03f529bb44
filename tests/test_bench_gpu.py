"""bench.py driver contract on the GPU box: one JSON line with the required keys, whole-job
value consistent with steps x tokens / time, for 1 rank and for a 2-rank rehearsal (gloo, both
ranks on cuda:0) of the multi-GPU flow (judge on rank 0, gather, max-over-ranks timing)."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _check(line, n_gpus, steps, warmup, max_tokens, judge):
    d = json.loads(line)
    assert KEYS <= set(d), set(d) ^ KEYS
    assert d["n_gpus"] == n_gpus and d["steps"] == steps and d["warmup"] == warmup
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "bf16"
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(d["config"])
    tokens = n_gpus * max_tokens + (max_tokens if judge else 0)
    assert abs(d["value"] - tokens * steps / (d["ms_per_step"] * steps / 1000)) < 0.02 * d["value"]
    return d


def test_bench_json_contract_1gpu(cuda):
    r = subprocess.run([sys.executable, "bench.py", "--model", "llama-small", "--judge", "llama-small", "--steps", "2",
                        "--warmup", "1", "--max-tokens", "48", "--results-dir", ""], cwd=ROOT, capture_output=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.strip()]
    assert len(lines) == 1
    _check(lines[0], 1, 2, 1, 48, judge=False)


def test_bench_two_rank_rehearsal(cuda):
    env = dict(os.environ, LLMC_BENCH_BACKEND="gloo", LLMC_BENCH_SAME_GPU="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29631", "bench.py", "--gpus", "2",
                        "--model", "llama-small", "--judge", "llama-small", "--steps", "1", "--warmup", "1",
                        "--max-tokens", "32", "--results-dir", ""], cwd=ROOT, capture_output=True, timeout=600,
                       env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = _check(lines[0], 2, 1, 1, 32, judge=True)
    assert d["extra"]["judge_prompt_tokens"] > 0
