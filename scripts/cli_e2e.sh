#!/bin/bash
# End-to-end CLI measurement on the GPU box: N local Llama-3-8B replicas + judge through the real
# llm-consensus entry point (worker processes, placement, streaming, incremental judge session).
# usage: bash scripts/cli_e2e.sh <tag> <n_models> <max_tokens> [extra CLI flags...]
set -e
tag=$1; n=$2; mt=$3; shift 3
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$root/gpurun_out/$tag"
models=$(python3 -c "print(','.join(f'llama-3-8b@{i}' for i in range($n)))")
t0=$(date +%s.%N)
timeout -k 10 900 python3 -m llm_consensus_amd --models "$models" --judge llama-3-8b@judge --max-tokens "$mt" \
  --data-dir "$root/gpurun_out/$tag/data" --trace -q "$@" \
  "Compare three sorting algorithms and recommend one for nearly-sorted data." \
  > "$root/gpurun_out/$tag/stdout.txt" 2> "$root/gpurun_out/$tag/stderr.txt"
t1=$(date +%s.%N)
python3 - "$root/gpurun_out/$tag" "$t0" "$t1" <<'PY'
import glob, json, os, sys
d, t0, t1 = sys.argv[1], float(sys.argv[2]), float(sys.argv[3])
run = sorted(glob.glob(os.path.join(d, "data", "*")))[-1]
res = json.load(open(os.path.join(run, "result.json")))
tr = json.load(open(os.path.join(run, "trace.json")))
lat = {r["model"]: r["latency_ms"] for r in res["responses"]}
print(json.dumps({"wall_s_incl_startup": round(t1 - t0, 2), "per_model_latency_ms": lat,
                  "n_responses": len(res["responses"]), "consensus_chars": len(res["consensus"]),
                  "trace_events": len(tr["traceEvents"])}))
PY
