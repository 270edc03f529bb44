# A/B: the fused attention + o_proj with the same-XCD L2 copy of the attention partials (mode 7,
# the default) vs without it (mode 39 = 7 | bit 5); lone 8B engine, alternating
for m in 7 39 7 39; do
  LLMC_ATTN_OPROJ=all LLMC_ATTN_OPROJ_MODE=$m timeout -k 10 200 python -u scripts/tp_shard_decode.py --tp 1 \
    --ctx 2048,9000 --tokens 256 | sed -u "s/^/mode=$m /" || exit $?
done
