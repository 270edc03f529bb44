# A/B: the Mixtral decode router folded into the fused attention + o_proj launch (LLMC_AO_ROUTER=1)
# vs its own launch (=0); the responder placement's lone-engine forms (LLMC_ATTN_OPROJ=all)
for v in 0 1 0 1; do
  LLMC_ATTN_OPROJ=all LLMC_AO_ROUTER=$v timeout -k 10 300 python -u scripts/tp_shard_decode.py --model mixtral-8x7b \
    --tp 1 --ctx 2048,9000 --tokens 256 | sed -u "s/^/ao_router=$v /" || exit $?
done
