# A/B of the lone engine's Infinity-Cache prefetch of the gate_up weights beside the fused attention launch
for cfg in "0 64" "32 64" "64 64" "64 128" "96 128"; do
  set -- $cfg
  LLMC_ATTN_OPROJ=all LLMC_PREFETCH_MB=$1 LLMC_PREFETCH_BLOCKS=$2 timeout -k 10 200 python -u scripts/tp_shard_decode.py --tp 1 --ctx 2048,9000 --tokens 256 | sed -u "s/^/pf=$1MB blocks=$2 /" || exit $?
done
