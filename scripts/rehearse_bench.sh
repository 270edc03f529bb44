#!/bin/bash
# Multi-rank bench flow rehearsed on ONE GPU (gloo bootstrap, every rank on cuda:0): exercises the
# judge-TP path (custom IPC all-reduce inside captured decode graphs, gloo for prefill-sized
# all-reduces) that the driver's N-GPU runs take over RCCL. Usage: rehearse_bench.sh NRANKS [bench args]
set -euo pipefail
N=${1:-2}; shift || true
export LLMC_BENCH_BACKEND=gloo LLMC_BENCH_SAME_GPU=1
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
  --master-port "${PORT:-29641}" bench.py --gpus "$N" --results-dir "" "$@"
