# Prefill GEMM counters (ours vs hipBLASLt on the gate_up shape, scripts/gemm_pmc_probe.py), one
# counter group per rocprofv3 run, then the prefill microbenchmark timings and the 33k-token judge
# prompt prefill. usage: gpurun -- bash scripts/gpu/pmc_gemm.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-pmcg}
mkdir -p $R/gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/ga -o ga -- python3 $R/scripts/gemm_pmc_probe.py > $R/gpurun_out/$tag/a.log 2>&1 && \
python3 $R/scripts/pmc_summary.py $(find /tmp/ga -name "*counter_collection.csv" | head -1) > $R/gpurun_out/$tag/a.md && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/gb -o gb -- python3 $R/scripts/gemm_pmc_probe.py > $R/gpurun_out/$tag/b.log 2>&1 && \
python3 $R/scripts/pmc_summary.py $(find /tmp/gb -name "*counter_collection.csv" | head -1) > $R/gpurun_out/$tag/b.md && \
cd $R && timeout -k 10 300 python3 -u scripts/microbench_kernels.py prefill > gpurun_out/$tag/prefill.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/tp_shard_decode.py --tp 1,8 --ctx 33000 --tokens 64 > gpurun_out/$tag/p33k.log 2>&1
