# A/B: 14-wave GEMV blocks for paired outputs (a TP=8 / TP=4 rank's gate_up: 256 / 512 blocks) vs
# 16-wave (224 / 448)
for v in 1 0 1 0; do
  if [ $v = 1 ]; then export LLMC_GEMV_NO_W14=1; else unset LLMC_GEMV_NO_W14; fi
  timeout -k 10 200 python -u scripts/tp_shard_decode.py --tp 8,4 --ctx 2048 --tokens 256 \
    | sed -u "s/^/no_w14=$v /" || exit $?
done
