set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LLMC_BENCH_BACKEND=gloo LLMC_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29633 bench.py --gpus 4 --config 5 --shapes tiny --steps 1 --warmup 0 --max-tokens 24 --results-dir "" > gpurun_out/r2_cfg5.log 2>&1
echo "cfg5 rc=$?"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_bench_gpu.py::test_bench_config5_rehearsal > gpurun_out/r2_full_pytest.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/r2_full_bench.log 2>&1 && \
bash scripts/prof_bench.sh r2_full_prof --steps 1 --warmup 0 --max-tokens 1024
