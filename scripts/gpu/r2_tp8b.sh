set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attn_decode" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_tp8b_tests.log 2>&1 && \
bash scripts/prof_tp_shard.sh r2_tp8b_33k --tp 8 --ctx 33000 --tokens 512 && \
timeout -k 10 300 python scripts/tp_shard_decode.py --tp 1,2,4,8 --ctx 2048,33000 > gpurun_out/r2_tp_shards.log 2>&1 && \
bash scripts/prof_decode.sh r2_dec13k_e --prompt 13500 --ctx 20480 --tokens 512
