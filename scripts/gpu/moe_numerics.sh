# MoE grouped GEMM (256 pipeline + SiLU epilogue) tests and microbench, full-size numerics tests,
# and a rocprofv3 kernel-stats profile of an 8k-token Mixtral prefill.
# usage: gpurun --timeout 1100 -- bash scripts/gpu/moe_numerics.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-moe}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "moe" -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_moe_tests.log 2>&1 && \
timeout -k 10 300 python scripts/microbench_kernels.py moe > gpurun_out/${tag}_moe_bench.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_numerics_full_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${tag}_numerics.log 2>&1 && \
bash scripts/prof_decode.sh ${tag}_mixtral_8k --model mixtral-8x7b --prompt 8192 --ctx 8704 --tokens 64
