# The driver's exact round-end command on the current tree, timed (must finish well inside 600 s).
cd $GRAFT_REPO_ROOT
tag=${1:-r4drv}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
start=$(date +%s)
step bench 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
echo "wall $(( $(date +%s) - start )) s" | tee -a gpurun_out/${tag}_steps.log
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
