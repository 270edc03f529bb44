# A/B on one box: the round-3 tree (ab_r3/, built in-tree) vs this tree, engine bench 2 timed rounds each.
cd $GRAFT_REPO_ROOT
tag=${1:-r4ab2}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step new1 300 python -u bench.py --steps 2 --warmup 1
step old1 300 bash -c "cd ab_r3 && python -u bench.py --steps 2 --warmup 1"
step new2 300 python -u bench.py --steps 2 --warmup 1
