# Round 4: attn_oproj with the head's merger requesting its own weight tile after the merge
# (mode 3) vs late weights (mode 1): correctness, microbenchmark, phase timeline, decode step.
cd $GRAFT_REPO_ROOT
tag=${1:-r4aod}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step pytest 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attn_oproj_gpu.py
step micro 300 python -u scripts/microbench_kernels.py attn-oproj
step tl 120 env AO_MODES=1,3 python -u scripts/ao_timeline.py 2048 9000
step dec1 200 env LLMC_ATTN_OPROJ_MODE=1 python -u scripts/tp_shard_decode.py --tp 1 --ctx 9000 --tokens 256
step dec3 200 env LLMC_ATTN_OPROJ_MODE=3 python -u scripts/tp_shard_decode.py --tp 1 --ctx 9000 --tokens 256
step dec1b 200 env LLMC_ATTN_OPROJ_MODE=1 python -u scripts/tp_shard_decode.py --tp 1 --ctx 9000 --tokens 256
step dec3b 200 env LLMC_ATTN_OPROJ_MODE=3 python -u scripts/tp_shard_decode.py --tp 1 --ctx 9000 --tokens 256
