#!/bin/bash
# usage (on the GPU box): bash scripts/prof_ep.sh <tag>
# rocprofv3 kernel stats of the expert-parallel prefill (scripts/ep_prefill_trace.py), one profiler
# per rank process (no process spawned under the profiler) -> gpurun_out/<tag>_r{0,1}_kernel_stats.md
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pb_$tag
port=$(python3 -c "import socket; s=socket.socket(); s.bind(('127.0.0.1',0)); print(s.getsockname()[1])")
for r in 0 1; do
  EP_RANK=$r EP_PORT=$port timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pb_$tag/r$r -o run -- \
    python3 "$root/scripts/ep_prefill_trace.py" > "$root/gpurun_out/${tag}_r$r.log" 2>&1 &
done
rc=0
for j in $(jobs -p); do wait $j || rc=$?; done
for r in 0 1; do
  f=$(find /tmp/pb_$tag/r$r -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$root/gpurun_out/${tag}_r${r}_kernel_stats.csv" && \
    python3 "$root/scripts/kstats.py" "$f" 60 > "$root/gpurun_out/${tag}_r${r}_kernel_stats.md"
done
exit $rc
