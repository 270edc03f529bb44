# A/B: cross-lane reductions by DPP / v_permlane*_swap (new library) vs ds_bpermute (abso/old_llmc_hip.so,
# built from the parent commit). The two libraries swap in place between runs.
L=llm_consensus_amd/_lib/_llmc_hip.cpython-310-x86_64-linux-gnu.so
cp $L abso/new_llmc_hip.so
run() {
  timeout -k 10 300 python -u scripts/tp_shard_decode.py --tp 1 --ctx 2048,9000 --tokens 256 | sed -u "s/^/$1 /" || return $?
  timeout -k 10 300 python -u scripts/tp_shard_decode.py --model phi-3-mini --tp 1 --ctx 2048 --tokens 256 | sed -u "s/^/$1 /" || return $?
}
for v in new old new old; do
  cp abso/${v}_llmc_hip.so $L || exit 1
  run $v || exit $?
done
cp abso/new_llmc_hip.so $L
