# Round 4 validation on the final tree: the GPU test suite, smoke(), and the driver's exact bench
# command (timed; it must finish well inside its 600 s).
cd $GRAFT_REPO_ROOT
tag=${1:-r4fin}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step pytest 600 python -u -m pytest tests/ -m gpu -q -rs --timeout 200 --timeout-method thread
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
start=$(date +%s)
step bench 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
echo "bench wall $(( $(date +%s) - start )) s" | tee -a gpurun_out/${tag}_steps.log
