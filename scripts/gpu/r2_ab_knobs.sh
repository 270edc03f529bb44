# A/B of launch knobs on a short bench round (3 x 8B responders + 8B judge, 1024 tokens): decode
# steps per graph replay (8 vs 16) and hardware queues per process (4 = HIP default vs 8)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python bench.py --results-dir '' --steps 2 --warmup 1 --max-tokens 1024 --warmup-tokens 256"
for i in 1 2; do
  timeout -k 10 240 bash -c "$B" > gpurun_out/ab_base_$i.log 2>&1 && \
  timeout -k 10 240 bash -c "$B --steps-per-graph 16" > gpurun_out/ab_spg16_$i.log 2>&1 && \
  timeout -k 10 240 bash -c "GPU_MAX_HW_QUEUES=8 $B" > gpurun_out/ab_hwq8_$i.log 2>&1 || exit 1
done
