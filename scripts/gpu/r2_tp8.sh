set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/prof_tp_shard.sh r2_tp8_33k --tp 8 --ctx 33000 --tokens 512
