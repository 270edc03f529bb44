set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_tp_gpu.py tests/test_bench_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_rccl.log 2>&1
