set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_tp_gpu.py tests/test_bench_gpu.py tests/test_custom_ar_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_tp3.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_full_pytest.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/r2_full_bench.log 2>&1 && \
bash scripts/prof_bench.sh r2_full_prof --steps 1 --warmup 0 --max-tokens 1024
