# consensus server with a Mixtral-8x7B responder: batched MoE decode (pairs grouped by expert)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/serve_bench.py --models mixtral-8x7b@0,llama-3-8b@1 --judge llama-3-8b@judge --concurrency 1,4,16 --requests 16 --max-tokens 256 > gpurun_out/r2_serve_moe.log 2>&1
