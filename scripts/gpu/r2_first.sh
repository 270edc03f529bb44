set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 2 --warmup 1 --models-per-gpu 3 > gpurun_out/r2_bench_mpg3.log 2>&1 && \
bash scripts/prof_bench.sh r2_prof_mpg3 --steps 1 --warmup 0 --models-per-gpu 3 --max-tokens 1024
