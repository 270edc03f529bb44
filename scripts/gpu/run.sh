# Generic GPU step runner (replaces the per-experiment one-off wrappers): each argument is one step
# "name|seconds|command ...", run under `timeout -k 10 <seconds>` with its output in
# gpurun_out/<tag>_<name>.log. A GPU fault, abort, segfault or time limit ends the script there
# (steps.sh); other failures are recorded and the next step runs.
# usage: gpurun --timeout N -- bash scripts/gpu/run.sh <tag> 'tests|400|python -u -m pytest tests/x.py -x -q' \
#            'decode|300|python -u scripts/tp_shard_decode.py --tp 1 --ctx 2048,9000 --tokens 256'
cd $GRAFT_REPO_ROOT
tag=$1; shift
mkdir -p gpurun_out
source scripts/gpu/steps.sh
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}
  secs=${rest%%|*}; cmd=${rest#*|}
  step "$name" "$secs" bash -c "$cmd"
done
grep -h "ms/token" gpurun_out/${tag}_*.log 2>/dev/null | head -40
exit 0
