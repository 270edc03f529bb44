# round-2 final validation: full GPU suite, smoke, driver-style bench, kernel stats of a bench round
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_final_pytest.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2_final_smoke.log 2>&1 && \
timeout -k 10 700 python bench.py --gpus 1 --steps 3 --warmup 2 > gpurun_out/r2_final_bench.log 2>&1
