# Consensus server throughput at 1 / 4 / 8 / 16 concurrent requests (batched decode).
# usage: gpurun -- bash scripts/gpu/serve.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/serve_bench.py --concurrency 1,4,8,16 --requests 16 --max-tokens 512 > gpurun_out/${1:-serve}.log 2>&1
