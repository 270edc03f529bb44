# the two-token-group GEMV tests against library builds: with the MFMA GEMV's norm sums by
# permlane swaps (nop) and with that one kernel back on ds_bpermute (nomfma)
L=llm_consensus_amd/_lib/_llmc_hip.cpython-310-x86_64-linux-gnu.so
cp $L abso/cur_llmc_hip.so
for v in nop nomfma nomfma; do
  cp abso/${v}_llmc_hip.so $L || exit 1
  echo "== $v"
  timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -q -k "batched_decode_rows or gemv_qkv_rope" --timeout 150 --timeout-method thread 2>&1 | grep -E "passed|failed" || true
done
cp abso/cur_llmc_hip.so $L
