set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attn_decode" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_attn7_tests.log 2>&1 && \
timeout -k 10 500 python scripts/microbench_kernels.py attn > gpurun_out/r2_attn7_micro.log 2>&1 && \
bash scripts/prof_decode.sh r2_dec13k_f --prompt 13500 --ctx 20480 --tokens 512
