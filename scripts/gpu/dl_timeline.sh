# Fused decode-layer task timelines (scripts/dl_timeline.py) at 2k and 13.5k context.
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-dlt}
mkdir -p gpurun_out
timeout -k 10 200 python scripts/dl_timeline.py --ctx 2048 > gpurun_out/${tag}_2k.log 2>&1 && \
timeout -k 10 200 python scripts/dl_timeline.py --ctx 13500 > gpurun_out/${tag}_13k.log 2>&1
