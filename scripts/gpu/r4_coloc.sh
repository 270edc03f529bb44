# Round 4: K engines sharing one GPU, each a TP=t shard of Llama-3-8B (scripts/colocated_shards.py):
# the compute side of placing every responder tensor-parallel over a GPU pair at N >= 4.
cd $GRAFT_REPO_ROOT
tag=${1:-r4coloc}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step k1t1 200 python -u scripts/colocated_shards.py --k 1 --tp 1
step k2t2 200 python -u scripts/colocated_shards.py --k 2 --tp 2
step k2t1 200 python -u scripts/colocated_shards.py --k 2 --tp 1
step k3t1 200 python -u scripts/colocated_shards.py --k 3 --tp 1
step k4t4 200 python -u scripts/colocated_shards.py --k 4 --tp 4
