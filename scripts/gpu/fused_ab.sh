# Fused decode layer: correctness tests, task timelines, 8B decode A/B vs the five-kernel step.
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-fab}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "fused" -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 && \
timeout -k 10 200 python scripts/dl_timeline.py --ctx 2048 > gpurun_out/${tag}_tl2k.log 2>&1 && \
timeout -k 10 200 python scripts/dl_timeline.py --ctx 13500 > gpurun_out/${tag}_tl13k.log 2>&1 && \
timeout -k 10 200 python scripts/profile_decode.py --prompt 2048 --ctx 8192 --tokens 512 --fused-layer 0 > gpurun_out/${tag}_dec2k_5k.log 2>&1 && \
timeout -k 10 200 python scripts/profile_decode.py --prompt 2048 --ctx 8192 --tokens 512 --fused-layer 1 > gpurun_out/${tag}_dec2k_fused.log 2>&1
