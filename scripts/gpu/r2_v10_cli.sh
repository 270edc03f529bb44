set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/cli_e2e.sh r2_v10_cli 3 4096 > gpurun_out/r2_v10_cli.log 2>&1
