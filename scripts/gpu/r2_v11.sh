# torch-free GPU count in the driver: test against the HIP runtime, then the CLI end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_placement.py tests/test_cli_local.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r2_v11_tests.log 2>&1 && \
bash scripts/cli_e2e.sh r2_v11_cli 3 4096 > gpurun_out/r2_v11_cli.log 2>&1
