# rocprofv3 kernel stats of the 8B decode at 9k keys: this tree's library vs the parent's
# (abso/old_llmc_hip.so, ds_bpermute reductions), swapped in place
L=llm_consensus_amd/_lib/_llmc_hip.cpython-310-x86_64-linux-gnu.so
cp $L abso/new_llmc_hip.so
for v in new old; do
  cp abso/${v}_llmc_hip.so $L || exit 1
  bash scripts/prof_decode.sh r6lx_prof_$v --ctx 9000 --tokens 128 || exit $?
done
cp abso/new_llmc_hip.so $L
