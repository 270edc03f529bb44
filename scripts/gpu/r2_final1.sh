set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_final1_pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_final1_smoke.log 2>&1 && \
timeout -k 10 500 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/r2_final1_bench.log 2>&1 && \
bash scripts/prof_bench.sh r2_final1_prof --steps 1 --warmup 0 --max-tokens 1024
