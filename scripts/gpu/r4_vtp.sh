# Round 4: the 8B judge as TP=2 over two CU-partitioned halves of ONE GPU (2 rank processes, fused
# all-reduce) against the TP=1 engine, at the N=1 bench judge's contexts.
cd $GRAFT_REPO_ROOT
tag=${1:-r4vtp}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step tp1 300 python -u scripts/tp_rehearsal.py --shape-tp 1 --world 1 --ctx 7500 --tokens 256 --fused-ar 0
step vtp2 300 python -u scripts/tp_rehearsal.py --shape-tp 2 --world 2 --ctx 7500 --tokens 256 --fused-ar 1
step vtp2s 300 python -u scripts/tp_rehearsal.py --shape-tp 2 --world 2 --ctx 7500 --tokens 256 --fused-ar 0
step vtp4 300 python -u scripts/tp_rehearsal.py --shape-tp 4 --world 4 --ctx 7500 --tokens 256 --fused-ar 1
