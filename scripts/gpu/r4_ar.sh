# Round 4: push-granule one-shot collectives and the fused row-parallel GEMV all-reduce (EPI_AR):
# GPU test suite, standalone all-reduce latency (ranks sharing one GPU), TP=8-shaped decode
# rehearsed over 2 CU-partitioned ranks with and without the fused epilogue, and the shard alone.
# usage: gpurun --timeout 1100 -- bash scripts/gpu/r4_ar.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-r4ar}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q -rs --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 && \
timeout -k 10 150 python -u scripts/car_latency.py --world 2,4 > gpurun_out/${tag}_carlat.log 2>&1 && \
timeout -k 10 200 python -u scripts/tp_rehearsal.py --shape-tp 8 --world 2 --fused-ar 0 > gpurun_out/${tag}_reh.log 2>&1 && \
timeout -k 10 200 python -u scripts/tp_rehearsal.py --shape-tp 8 --world 2 --fused-ar 1 >> gpurun_out/${tag}_reh.log 2>&1 && \
timeout -k 10 200 python -u scripts/tp_shard_decode.py --tp 8 --ctx 2048 --tokens 256 > gpurun_out/${tag}_shard.log 2>&1 && \
timeout -k 10 240 python -u scripts/microbench_kernels.py prefill > gpurun_out/${tag}_prefill_gemm.log 2>&1
