set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/cli_e2e.sh r2_cli3 3 4096 > gpurun_out/r2_cli3.log 2>&1 && \
timeout -k 10 600 python scripts/serve_bench.py > gpurun_out/r2_serve.log 2>&1
