# A/B: the o_proj (+ TP all-reduce) inside the one-launch qkv + attention (the o-role) vs the o GEMV after it
for v in 0 1 0 1; do
  LLMC_QKV_ATTN_O=$v timeout -k 10 250 python -u scripts/tp_shard_decode.py --tp 8,4 --ctx 2048,16000 --tokens 256 | sed -u "s/^/qa_o=$v /" || exit $?
done
for v in 0 1; do
  LLMC_QKV_ATTN_O=$v timeout -k 10 250 python -u scripts/tp_rehearsal.py --shape-tp 8 --world 2 --ctx 2048 --tokens 256 --fused-ar 1 | sed -u "s/^/qa_o=$v /" || exit $?
done
