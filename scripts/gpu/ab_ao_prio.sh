# A/B: the fused attention + o_proj launch with the control waves at a higher issue priority (mode bit 4)
for m in 7 23 7 23; do
  LLMC_ATTN_OPROJ=all LLMC_ATTN_OPROJ_MODE=$m timeout -k 10 200 python -u scripts/tp_shard_decode.py --tp 1 --ctx 2048,9000 --tokens 256 | sed -u "s/^/mode=$m /" || exit $?
done
LLMC_ATTN_OPROJ=all LLMC_ATTN_OPROJ_MODE=23 timeout -k 10 200 python -u scripts/profile_decode.py --model mixtral-8x7b --prompt 2048 --tokens 256 --ctx 4096 | sed -u "s/^/mode=23 /"
