set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_mix3_pytest.log 2>&1 && \
bash scripts/prof_decode.sh r2_dec2k_d --prompt 2048 --ctx 8192 --tokens 512 && \
bash scripts/prof_decode.sh r2_dec13k_d --prompt 13500 --ctx 20480 --tokens 512 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/r2_mix3_bench.log 2>&1
