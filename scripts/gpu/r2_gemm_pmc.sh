set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc1 -o p1 -- python3 $R/scripts/gemm_pmc_probe.py > $R/gpurun_out/pmc/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_COUNT --output-format csv -d /tmp/pmc2 -o p2 -- python3 $R/scripts/gemm_pmc_probe.py > $R/gpurun_out/pmc/p2.log 2>&1 && \
cp $(find /tmp/pmc1 -name "*counter_collection.csv" | head -1) $R/gpurun_out/pmc/p1.csv && \
cp $(find /tmp/pmc2 -name "*counter_collection.csv" | head -1) $R/gpurun_out/pmc/p2.csv
