#!/bin/bash
# usage (on the GPU box): bash scripts/prof_tp_rehearsal.sh <tag> [tp_rehearsal.py args...]
# rocprofv3 kernel stats of a TP group rehearsed on one GPU (scripts/tp_rehearsal.py: rank processes
# on disjoint CUs) -> gpurun_out/<tag>_kernel_stats.{csv,md}: which collectives the decode runs
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pr_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pr_$tag -o run -- \
  python3 "$root/scripts/tp_rehearsal.py" "$@" > "$root/gpurun_out/${tag}.log" 2>&1
for f in $(find /tmp/pr_$tag -name "run_kernel_stats.csv"); do
  n=$(echo "$f" | md5sum | cut -c1-6)
  cp "$f" "$root/gpurun_out/${tag}_${n}_kernel_stats.csv"
  python3 "$root/scripts/kstats.py" "$f" 25 > "$root/gpurun_out/${tag}_${n}_kernel_stats.md"
done
grep -E "ms/token" "$root/gpurun_out/${tag}.log"
