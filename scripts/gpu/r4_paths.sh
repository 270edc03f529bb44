# Round 4: the product path vs the engine path at the bench configuration (2 timed rounds each), the
# --max-tokens 4096 secondary on the final tree, and a rocprofv3 table of the TP=8-shaped decode
# rehearsed over 2 CU-partitioned ranks (fused all-reduce epilogue: no standalone all-reduce
# launch in decode).
# usage: gpurun --timeout 1150 -- bash scripts/gpu/r4_paths.sh <tag>
cd $GRAFT_REPO_ROOT
tag=${1:-r4p}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step engine 260 python -u bench.py --steps 2 --warmup 1
step cli 320 python -u bench.py --path cli --steps 2 --warmup 1
step mt4096 300 python -u bench.py --steps 2 --warmup 1 --max-tokens 4096
step reh_k1 240 python -u scripts/tp_rehearsal.py --shape-tp 8 --world 2 --tokens 128 --reps 1 --trace-kernels 1
step reh_k0 240 python -u scripts/tp_rehearsal.py --shape-tp 8 --world 2 --tokens 128 --reps 1 --trace-kernels 1 --fused-ar 0
