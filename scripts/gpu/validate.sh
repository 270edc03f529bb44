# Full GPU validation of the tree: the GPU test suite, smoke(), and a short bench round.
# usage: gpurun --timeout 900 -- bash scripts/gpu/validate.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-val}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/${tag}_bench.log 2>&1
