set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_custom_ar_gpu.py tests/test_bench_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_tp_tests.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/r2_bench_default.log 2>&1
