# One rocprofv3 counter pass over the flash prefill at PMC_PREFILL tokens (default 2048,8192): MFMA
# busy / bf16 MOPs, VALU instructions, LDS activity and bank conflicts, waves, busy cycles.
# usage: gpurun -- bash scripts/gpu/pmc_prefill.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-pmcpf}
mkdir -p $R/gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp
export PMC_PREFILL=${PMC_PREFILL:-2048,8192} PMC_PREFILL_ONLY=1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/pf_$tag -o pf -- python3 $R/scripts/pmc_kernels.py > $R/gpurun_out/$tag/a.log 2>&1 && \
python3 $R/scripts/pmc_summary.py $(find /tmp/pf_$tag -name "*counter_collection.csv" | head -1) > $R/gpurun_out/$tag/a.md
