# Round 4: per-layer numerics at the judge context, the product path vs the engine path at the bench
# configuration (2 timed rounds each), and a rocprofv3 table of the TP=8-shaped decode rehearsed over 2
# CU-partitioned ranks (fused all-reduce epilogue: no standalone all-reduce launch in decode).
# usage: gpurun --timeout 1100 -- bash scripts/gpu/r4_paths.sh <tag>
cd $GRAFT_REPO_ROOT
tag=${1:-r4p}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step perlayer 300 python -u -m pytest tests/test_numerics_full_gpu.py -k per_layer -x -q -s --timeout 280 --timeout-method thread
step engine 240 python -u bench.py --steps 2 --warmup 1
step cli 300 python -u bench.py --path cli --steps 2 --warmup 1
step reh_prof 300 bash scripts/prof_tp_rehearsal.sh ${tag}_rehprof --shape-tp 8 --world 2 --tokens 128 --reps 1
