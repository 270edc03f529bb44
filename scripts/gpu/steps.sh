# Helper for scripts/gpu/*.sh: `step <name> <timeout-s> <command...>` runs one GPU step under its own
# time limit with output in gpurun_out/<tag>_<name>.log. A failing step (tests that fail) does not
# stop the script; a time limit, an abort or a crash (exit status 124, 134, 137, 139 or > 128) ends
# it there, so nothing more runs on a GPU that may be in a bad state.
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_${name}.log" 2>&1
  local rc=$?
  echo "[step] $name rc=$rc" | tee -a "gpurun_out/${tag}_steps.log"
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "[step] $name ended the script (rc=$rc)" | tee -a "gpurun_out/${tag}_steps.log"
    exit $rc
  fi
  return 0
}
