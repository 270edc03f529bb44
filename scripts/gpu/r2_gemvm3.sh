# MFMA decode form variants: numerics of every pinned form, then the per-shape sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "gemvm or batched or qkv_rope or fused_norm" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gemvm3_tests.log 2>&1 && \
timeout -k 10 600 python -u scripts/microbench_kernels.py gemvm-forms > gpurun_out/r2_gemvm3_forms.log 2>&1
