cd $GRAFT_REPO_ROOT
tag=${1:-r4tpchk}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step tests 400 python -u -m pytest tests/test_tp_gpu.py tests/test_custom_ar_gpu.py tests/test_bench_gpu.py tests/test_qkv_attn_gpu.py -x -q --timeout 200 --timeout-method thread
step n2 300 env PORT=29675 bash scripts/rehearse_bench.sh 2 --steps 1 --warmup 1 --max-tokens 128 --judge-max-tokens 16
