# Fused decode layer: its GPU tests, then 8B batch-1 decode A/B (five kernels vs one fused launch
# per layer) at 2k and 13.5k context under rocprofv3 kernel stats.
# usage: gpurun --timeout 1100 -- bash scripts/gpu/fused_layer.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-fl}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "fused or oracle or graph" -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 && \
timeout -k 10 200 python scripts/profile_decode.py --prompt 2048 --ctx 8192 --tokens 512 --fused-layer 0 > gpurun_out/${tag}_dec2k_5k.log 2>&1 && \
timeout -k 10 200 python scripts/profile_decode.py --prompt 2048 --ctx 8192 --tokens 512 --fused-layer 1 > gpurun_out/${tag}_dec2k_fused.log 2>&1 && \
timeout -k 10 200 python scripts/profile_decode.py --prompt 13500 --ctx 20480 --tokens 512 --fused-layer 0 > gpurun_out/${tag}_dec13k_5k.log 2>&1 && \
timeout -k 10 200 python scripts/profile_decode.py --prompt 13500 --ctx 20480 --tokens 512 --fused-layer 1 > gpurun_out/${tag}_dec13k_fused.log 2>&1 && \
bash scripts/prof_decode.sh ${tag}_dec2k_fused_prof --prompt 2048 --ctx 8192 --tokens 512 --fused-layer 1
