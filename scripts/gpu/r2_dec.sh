set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/prof_decode.sh r2_dec2k --prompt 2048 --ctx 8192 --tokens 512 && \
bash scripts/prof_decode.sh r2_dec13k --prompt 13500 --ctx 20480 --tokens 512 && \
timeout -k 10 300 python scripts/microbench_kernels.py attn > gpurun_out/r2_attn3_microbench.log 2>&1
