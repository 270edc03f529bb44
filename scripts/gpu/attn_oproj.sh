# Fused decode attention + o_proj (csrc/kernels/attn_oproj.hip): its GPU tests, the microbenchmark
# against the two launches, and the 8B decode step with the fused launch on / off.
# usage: gpurun --timeout 900 -- bash scripts/gpu/attn_oproj.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-ao}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attn_oproj_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/microbench_kernels.py attn-oproj > gpurun_out/${tag}_micro.log 2>&1 || exit $?
for v in 1 0; do
  LLMC_ATTN_OPROJ=$v timeout -k 10 240 python -u scripts/tp_shard_decode.py --tp 1 --ctx 2048,7600,9000,13000 \
    --tokens 256 > gpurun_out/${tag}_decode_ao$v.log 2>&1 || exit $?
done
grep -H "ms/token" gpurun_out/${tag}_decode_ao*.log
