# A/B: the gate_up GEMV's SiLU epilogue with both pair rows in one wave (RPW 2) vs the LDS pair
# exchange (RPW 1): kernel microbench, then the lone 8B decode and Phi-3
LLMC_GEMV_SILU_RPW1=1 timeout -k 10 150 python -u scripts/microbench_kernels.py gemv | sed -u "s/^/rpw1 /" || exit $?
timeout -k 10 150 python -u scripts/microbench_kernels.py gemv | sed -u "s/^/rpw2 /" || exit $?
for v in 1 0 1 0; do
  if [ $v = 1 ]; then export LLMC_GEMV_SILU_RPW1=1; else unset LLMC_GEMV_SILU_RPW1; fi
  LLMC_ATTN_OPROJ=all timeout -k 10 200 python -u scripts/tp_shard_decode.py --tp 1 --ctx 2048,9000 --tokens 256 \
    | sed -u "s/^/silu_rpw1=$v /" || exit $?
done
