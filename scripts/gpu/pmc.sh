# rocprofv3 counter passes over scripts/pmc_kernels.py, one counter group per run (never combined
# with trace domains). usage: gpurun -- bash scripts/gpu/pmc.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-pmc}
mkdir -p $R/gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/scripts/pmc_kernels.py > $R/gpurun_out/$tag/plain.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/pa -o pa -- python3 $R/scripts/pmc_kernels.py > $R/gpurun_out/$tag/a.log 2>&1 && \
python3 $R/scripts/pmc_summary.py $(find /tmp/pa -name "*counter_collection.csv" | head -1) > $R/gpurun_out/$tag/a.md && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pb -o pb -- python3 $R/scripts/pmc_kernels.py > $R/gpurun_out/$tag/b.log 2>&1 && \
python3 $R/scripts/pmc_summary.py $(find /tmp/pb -name "*counter_collection.csv" | head -1) > $R/gpurun_out/$tag/b.md && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d /tmp/pc -o pc -- python3 $R/scripts/pmc_kernels.py > $R/gpurun_out/$tag/c.log 2>&1 && \
python3 $R/scripts/pmc_summary.py $(find /tmp/pc -name "*counter_collection.csv" | head -1) > $R/gpurun_out/$tag/c.md
