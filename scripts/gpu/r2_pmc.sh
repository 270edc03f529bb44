# rocprofv3 counter passes over scripts/pmc_kernels.py, one counter group per run
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/scripts/pmc_kernels.py > $R/gpurun_out/pmc2/plain.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/pa -o pa -- python3 $R/scripts/pmc_kernels.py > $R/gpurun_out/pmc2/a.log 2>&1 && \
python3 $R/scripts/pmc_summary.py $(find /tmp/pa -name "*counter_collection.csv" | head -1) > $R/gpurun_out/pmc2/a.md && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pb -o pb -- python3 $R/scripts/pmc_kernels.py > $R/gpurun_out/pmc2/b.log 2>&1 && \
python3 $R/scripts/pmc_summary.py $(find /tmp/pb -name "*counter_collection.csv" | head -1) > $R/gpurun_out/pmc2/b.md && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d /tmp/pc -o pc -- python3 $R/scripts/pmc_kernels.py > $R/gpurun_out/pmc2/c.log 2>&1 && \
python3 $R/scripts/pmc_summary.py $(find /tmp/pc -name "*counter_collection.csv" | head -1) > $R/gpurun_out/pmc2/c.md && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt -o pt -- python3 $R/scripts/pmc_kernels.py > $R/gpurun_out/pmc2/t.log 2>&1 && \
python3 $R/scripts/kstats.py $(find /tmp/pt -name "pt_kernel_stats.csv" | head -1) 20 > $R/gpurun_out/pmc2/t.md
