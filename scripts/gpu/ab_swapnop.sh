# A/B: permlane swaps with 2 wait states before (new) vs 5 before and after (abso/old_llmc_hip.so)
L=llm_consensus_amd/_lib/_llmc_hip.cpython-310-x86_64-linux-gnu.so
cp $L abso/new_llmc_hip.so
for v in new old new old; do
  cp abso/${v}_llmc_hip.so $L || exit 1
  timeout -k 10 300 python -u scripts/tp_shard_decode.py --tp 1 --ctx 2048,9000 --tokens 256 | sed -u "s/^/$v /" || exit $?
done
cp abso/new_llmc_hip.so $L
