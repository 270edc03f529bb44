# Round-3 evidence pass: MoE grouped GEMM tests + microbench, full-size numerics tests, the new
# attention rounding test, Mixtral 8k prefill profile, and the per-rank shard profiles of configs 4/5.
# usage: gpurun --timeout 1150 -- bash scripts/gpu/r3_evidence.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-ev}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "moe or partial_rounding" -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_kernel_tests.log 2>&1 && \
timeout -k 10 240 python scripts/microbench_kernels.py moe > gpurun_out/${tag}_moe_bench.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_numerics_full_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${tag}_numerics.log 2>&1 && \
bash scripts/prof_decode.sh ${tag}_mixtral_8k --model mixtral-8x7b --prompt 8192 --ctx 8704 --tokens 64 && \
bash scripts/gpu/shards.sh ${tag}
