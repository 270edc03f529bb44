# Round 4: attn_oproj with whole o_proj rows per block (mode 7: no tile reduce) vs mode 3:
# correctness (the default-mode tests run under mode 7 too), microbenchmark, timeline, decode step.
cd $GRAFT_REPO_ROOT
tag=${1:-r4aofr}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step pytest 300 env LLMC_ATTN_OPROJ_MODE=7 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attn_oproj_gpu.py
step micro 300 python -u scripts/microbench_kernels.py attn-oproj
step tl 120 env AO_MODES=3,7 python -u scripts/ao_timeline.py 2048 9000
for ctx in 9000 7500; do
  step dec3_$ctx 200 env LLMC_ATTN_OPROJ_MODE=3 python -u scripts/tp_shard_decode.py --tp 1 --ctx $ctx --tokens 256
  step dec7_$ctx 200 env LLMC_ATTN_OPROJ_MODE=7 python -u scripts/tp_shard_decode.py --tp 1 --ctx $ctx --tokens 256
  step dec3b_$ctx 200 env LLMC_ATTN_OPROJ_MODE=3 python -u scripts/tp_shard_decode.py --tp 1 --ctx $ctx --tokens 256
  step dec7b_$ctx 200 env LLMC_ATTN_OPROJ_MODE=7 python -u scripts/tp_shard_decode.py --tp 1 --ctx $ctx --tokens 256
done
