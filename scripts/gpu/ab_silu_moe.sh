# A/B: Mixtral's expert gate_up with both SiLU pair rows in one wave vs the LDS pair exchange
for v in 1 0 1 0; do
  if [ $v = 1 ]; then export LLMC_GEMV_SILU_RPW1=1; else unset LLMC_GEMV_SILU_RPW1; fi
  LLMC_ATTN_OPROJ=all timeout -k 10 300 python -u scripts/tp_shard_decode.py --model mixtral-8x7b --tp 1 --ctx 2048 --tokens 256 \
    | sed -u "s/^/silu_rpw1=$v /" || exit $?
done
