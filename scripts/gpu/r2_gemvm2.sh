# full GPU suite after the batched-decode MFMA form + its microbenchmark
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_gemvm2_pytest.log 2>&1 && \
timeout -k 10 300 python -u scripts/microbench_kernels.py batched > gpurun_out/r2_gemvm2_bench.log 2>&1
