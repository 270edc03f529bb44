# Round 4: push-granule one-shot collectives and the fused row-parallel GEMV all-reduce (EPI_AR):
# GPU test suite, standalone all-reduce latency (ranks
# sharing one GPU), TP=8-shaped decode rehearsed over 2 CU-partitioned ranks with and without the
# fused epilogue, the shard alone, prefill GEMM and attention + o_proj microbenchmarks.
# usage: gpurun --timeout 1100 -- bash scripts/gpu/r4_ar.sh <tag>
cd $GRAFT_REPO_ROOT
tag=${1:-r4ar}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step pytest 600 python -u -m pytest tests/ -m gpu -q -rs --timeout 200 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step carlat 150 python -u scripts/car_latency.py --world 2,4
step reh0 200 python -u scripts/tp_rehearsal.py --shape-tp 8 --world 2 --fused-ar 0
step reh1 200 python -u scripts/tp_rehearsal.py --shape-tp 8 --world 2 --fused-ar 1
step shard 200 python -u scripts/tp_shard_decode.py --tp 8 --ctx 2048 --tokens 256
step attn_oproj 240 python -u scripts/microbench_kernels.py attn-oproj
step prefill_gemm 240 python -u scripts/microbench_kernels.py prefill
