# Second half of scripts/gpu/r3_evidence.sh: full-size numerics, Mixtral 8k prefill profile, shard profiles.
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-ev}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_numerics_full_gpu.py -v -s --timeout 400 --timeout-method thread > gpurun_out/${tag}_numerics.log 2>&1
rc=$?
# a failed assertion (1) still lets the profiles run; an abort, fault or time limit ends the call
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/prof_decode.sh ${tag}_mixtral_8k --model mixtral-8x7b --prompt 8192 --ctx 8704 --tokens 64 && \
bash scripts/gpu/shards.sh ${tag}
