# A/B of the next-layer Infinity-Cache prefetch on latency-bound TP shards (one rank alone)
for cfg in "0 64" "64 128" "64 256" "128 256"; do
  set -- $cfg
  LLMC_PREFETCH_NEXT_MB=$1 LLMC_PREFETCH_BLOCKS=$2 timeout -k 10 250 python -u scripts/tp_shard_decode.py --tp 8,4,2 --ctx 2048 --tokens 256 | sed -u "s/^/next=$1MB blocks=$2 /" || exit $?
done
for cfg in "0 64" "64 256"; do
  set -- $cfg
  LLMC_PREFETCH_NEXT_MB=$1 LLMC_PREFETCH_BLOCKS=$2 timeout -k 10 250 python -u scripts/tp_shard_decode.py --model llama-3-70b --tp 4 --ctx 2048 --tokens 256 | sed -u "s/^/next=$1MB blocks=$2 /" || exit $?
done
