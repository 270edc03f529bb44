for m in 7 15; do
  LLMC_ATTN_OPROJ=all LLMC_ATTN_OPROJ_MODE=$m timeout -k 10 200 python -u scripts/tp_shard_decode.py --tp 1 --ctx 2048,5000,9000 --tokens 256 | sed "s/^/mode=$m /" || exit $?
done
for m in 7 15; do
  LLMC_ATTN_OPROJ=all LLMC_ATTN_OPROJ_MODE=$m timeout -k 10 200 python -u scripts/profile_decode.py --model mixtral-8x7b --prompt 2048 --tokens 256 --ctx 4096 | sed "s/^/mode=$m /" || exit $?
done
