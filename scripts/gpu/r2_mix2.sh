set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attn_decode" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_mix2_tests.log 2>&1 && \
timeout -k 10 300 python scripts/microbench_kernels.py prefill > gpurun_out/r2_mix2_gemm.log 2>&1 && \
timeout -k 10 300 python scripts/microbench_kernels.py attn > gpurun_out/r2_mix2_attn.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/r2_mix2_bench.log 2>&1
