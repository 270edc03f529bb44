set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc3 -o p3 -- python3 $R/scripts/gemm_pmc_probe.py > $R/gpurun_out/pmc/p3.log 2>&1 && \
cp $(find /tmp/pmc3 -name "*counter_collection.csv" | head -1) $R/gpurun_out/pmc/p3.csv
