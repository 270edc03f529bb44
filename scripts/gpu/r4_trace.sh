# Round 4: which kernels a TP=8-shaped decode launches (2 CU-partitioned ranks, torch.profiler):
# fused all-reduce (no standalone car_* launches in decode) vs separate all-reduce launches.
cd $GRAFT_REPO_ROOT
tag=${1:-r4trace}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step k1 240 python -u scripts/tp_rehearsal.py --shape-tp 8 --world 2 --tokens 128 --reps 1 --trace-kernels 1
step k0 240 python -u scripts/tp_rehearsal.py --shape-tp 8 --world 2 --tokens 128 --reps 1 --trace-kernels 1 --fused-ar 0
