# A/B: geometries of Mixtral's fused expert down projection + combine
for g in default 512u4 1024u8 512u8 1024u2 default; do
  if [ $g = default ]; then unset LLMC_DC_GEOM; else export LLMC_DC_GEOM=$g; fi
  LLMC_ATTN_OPROJ=all timeout -k 10 300 python -u scripts/tp_shard_decode.py --model mixtral-8x7b --tp 1 --ctx 2048 --tokens 256 \
    | sed -u "s/^/dc=$g /" || exit $?
done
