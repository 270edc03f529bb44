# GPU validation of the tree: optional targeted tests first, then the whole GPU suite, smoke() and a
# short bench round. Every step under its own time limit, chained with && (stops at the first failure).
# usage: gpurun --timeout 1100 -- bash scripts/gpu/validate.sh <tag> [pytest targets for the first pass...]
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-val}; shift || true
mkdir -p gpurun_out
first=true
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -x -v --timeout 150 --timeout-method thread > gpurun_out/${tag}_first.log 2>&1 || first=false
fi
$first && \
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/${tag}_bench.log 2>&1
