# A/B of the SiLU RPW 2 form on the other shapes it takes: Phi-3-mini (16384 rows, 16 waves) and
# the 8B TP=4 rank (7168 rows, 14 waves); TP=8 (3584) keeps RPW 1
for v in 1 0 1 0; do
  if [ $v = 1 ]; then export LLMC_GEMV_SILU_RPW1=1; else unset LLMC_GEMV_SILU_RPW1; fi
  LLMC_ATTN_OPROJ=all timeout -k 10 200 python -u scripts/tp_shard_decode.py --model phi-3-mini --tp 1 --ctx 2048 --tokens 256 \
    | sed -u "s/^/silu_rpw1=$v /" || exit $?
  timeout -k 10 200 python -u scripts/tp_shard_decode.py --tp 4 --ctx 2048 --tokens 256 | sed -u "s/^/silu_rpw1=$v /" || exit $?
done
