set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_bench_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r2_bench2_tests.log 2>&1 && \
PORT=29657 timeout -k 20 900 bash scripts/rehearse_bench.sh 2 --steps 1 --warmup 0 --max-tokens 1024 > gpurun_out/r2_rehearse2.log 2>&1
