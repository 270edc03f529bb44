#!/bin/bash
# usage (GPU box): bash scripts/prof_bench.sh <tag> [bench.py args...]
# rocprofv3 kernel stats of one bench.py round (1 rank) -> gpurun_out/<tag>_kernel_stats.{csv,md}
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pb_$tag
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pb_$tag -o run -- \
  python3 "$root/bench.py" --results-dir "" "$@" > "$root/gpurun_out/${tag}.log" 2>&1
f=$(find /tmp/pb_$tag -name "run_kernel_stats.csv" | head -1)
cp "$f" "$root/gpurun_out/${tag}_kernel_stats.csv"
python3 "$root/scripts/kstats.py" "$f" 25 > "$root/gpurun_out/${tag}_kernel_stats.md"
