set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PORT=29655 timeout -k 20 1000 bash scripts/rehearse_bench.sh 8 --steps 1 --warmup 0 --max-tokens 1024 > gpurun_out/r2_rehearse8.log 2>&1
