set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attn_decode" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_attn5_tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_attn5_engine.log 2>&1 && \
timeout -k 10 300 python scripts/microbench_kernels.py attn > gpurun_out/r2_attn5_microbench.log 2>&1 && \
bash scripts/prof_decode.sh r2_dec2k_c --prompt 2048 --ctx 8192 --tokens 512 && \
bash scripts/prof_decode.sh r2_dec13k_c --prompt 13500 --ctx 20480 --tokens 512 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/r2_attn5_bench.log 2>&1
