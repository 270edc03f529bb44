# Round 4: 8B decode at ~9k keys after the attn_oproj merger-defers default (rocprofv3 kernel stats).
cd $GRAFT_REPO_ROOT
tag=${1:-r4aod_dec9k}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step prof 400 bash scripts/prof_decode.sh $tag --prompt 8704 --ctx 9400 --tokens 512
