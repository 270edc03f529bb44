# Un-profiled per-rank decode timings: one TP rank's shard alone on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-st}
mkdir -p gpurun_out
out=gpurun_out/${tag}_shards.log
: > $out
for spec in "llama-3-8b 1 2048,33000" "llama-3-8b 2 2048,33000" "llama-3-8b 4 2048,33000" "llama-3-8b 8 2048,33000" \
            "llama-3-70b 2 2048,16384" "llama-3-70b 4 2048,16384" "llama-3-70b 8 2048,16384"; do
  set -- $spec
  timeout -k 10 240 python -u scripts/tp_shard_decode.py --model $1 --tp $2 --ctx $3 --tokens 256 >> $out 2>&1 || exit $?
done
grep "ms/token" $out
