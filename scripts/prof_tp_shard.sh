#!/bin/bash
# usage (on the GPU box): bash scripts/prof_tp_shard.sh <tag> [tp_shard_decode.py args...]
# rocprofv3 kernel stats of one TP rank's Llama-3-8B shard decoding alone -> gpurun_out/<tag>_kernel_stats.{csv,md}
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pb_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pb_$tag -o run -- \
  python3 "$root/scripts/tp_shard_decode.py" "$@" > "$root/gpurun_out/${tag}.log" 2>&1
f=$(find /tmp/pb_$tag -name "run_kernel_stats.csv" | head -1)
cp "$f" "$root/gpurun_out/${tag}_kernel_stats.csv"
python3 "$root/scripts/kstats.py" "$f" 25 > "$root/gpurun_out/${tag}_kernel_stats.md"
grep -E "ms/token" "$root/gpurun_out/${tag}.log"
cat "$root/gpurun_out/${tag}_kernel_stats.md" | head -14
