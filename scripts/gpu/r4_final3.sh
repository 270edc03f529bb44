# Round 4: GPU suite on the final tree.
cd $GRAFT_REPO_ROOT
tag=${1:-r4fin3}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step pytest 600 python -u -m pytest tests/ -m gpu -q -rs --timeout 200 --timeout-method thread
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
