# A/B: 10-wave GEMV blocks for the 70B TP=4 rank's qkv (2560 x 8192: 256 blocks) vs 16-wave (160)
for v in 1 0 1 0; do
  if [ $v = 1 ]; then export LLMC_GEMV_NO_W10=1; else unset LLMC_GEMV_NO_W10; fi
  timeout -k 10 280 python -u scripts/tp_shard_decode.py --model llama-3-70b --tp 4 --ctx 2048 --tokens 128 \
    | sed -u "s/^/no_w10=$v /" || exit $?
done
