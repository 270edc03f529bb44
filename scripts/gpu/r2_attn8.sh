set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attn_decode" -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_attn8_tests.log 2>&1
