# Multi-rank bench flows (N = 2, 4, 8 ranks sharing one GPU, gloo bootstrap): checks the flow end to
# end; the timing says nothing about a multi-GPU node. usage: gpurun -- bash scripts/gpu/rehearse.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-reh}
mkdir -p gpurun_out
PORT=29661 timeout -k 20 300 bash scripts/rehearse_bench.sh 2 --steps 1 --warmup 1 --max-tokens 256 --judge-max-tokens 64 > gpurun_out/${tag}2.log 2>&1 && \
PORT=29662 timeout -k 20 300 bash scripts/rehearse_bench.sh 4 --steps 1 --warmup 0 --max-tokens 256 --judge-max-tokens 64 > gpurun_out/${tag}4.log 2>&1 && \
LLMC_BENCH_CU_SPLIT=1 PORT=29663 timeout -k 20 420 bash scripts/rehearse_bench.sh 8 --steps 1 --warmup 0 --max-tokens 256 --judge-max-tokens 32 > gpurun_out/${tag}8.log 2>&1
