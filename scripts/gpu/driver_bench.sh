# The driver's exact 1-GPU bench command under its 600-s limit, then the GPU test suite.
# usage: gpurun --timeout 1100 -- bash scripts/gpu/driver_bench.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-r3}
mkdir -p gpurun_out
start=$(date +%s.%N)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_driver_bench.out 2> gpurun_out/${tag}_driver_bench.err
rc=$?
end=$(date +%s.%N)
python3 -c "import sys; print({\"rc\": int(sys.argv[1]), \"wall_s\": round(float(sys.argv[3]) - float(sys.argv[2]), 1)})" $rc $start $end > gpurun_out/${tag}_driver_bench.wall
cat gpurun_out/${tag}_driver_bench.wall
[ $rc -eq 0 ] || exit $rc
if [ "${2:-}" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1
fi
