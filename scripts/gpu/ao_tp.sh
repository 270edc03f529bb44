# Fused attention + o_proj on one TP rank's shard (scripts/tp_shard_decode.py, no all-reduce): on in
# every bucket it covers (LLMC_ATTN_OPROJ=all), off (0), at the judge's contexts for N = 1/2/4/8.
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-aotp}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
for spec in "1 2048,9000" "2 8500,9400" "4 10500" "8 20000"; do
  set -- $spec
  for v in all 0; do
    echo "== tp=$1 LLMC_ATTN_OPROJ=$v" >> $out
    LLMC_ATTN_OPROJ=$v timeout -k 10 200 python -u scripts/tp_shard_decode.py --tp $1 --ctx $2 --tokens 256 >> $out 2>&1 || exit $?
  done
done
grep -E "^==|ms/token" $out
