# multi-rank bench flows (N = 2, 4, 8 ranks sharing one GPU, gloo bootstrap) on the final round-2 tree;
# short rounds: the timing says nothing about a multi-GPU node, the run checks the flow end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PORT=29661 timeout -k 20 300 bash scripts/rehearse_bench.sh 2 --steps 1 --warmup 0 --max-tokens 256 --judge-max-tokens 64 > gpurun_out/r2_reh2.log 2>&1 && \
PORT=29662 timeout -k 20 300 bash scripts/rehearse_bench.sh 4 --steps 1 --warmup 0 --max-tokens 256 --judge-max-tokens 64 > gpurun_out/r2_reh4.log 2>&1 && \
PORT=29663 timeout -k 20 420 bash scripts/rehearse_bench.sh 8 --steps 1 --warmup 0 --max-tokens 256 --judge-max-tokens 32 > gpurun_out/r2_reh8.log 2>&1
