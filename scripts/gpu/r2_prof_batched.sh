# 8B decode with 16 rows per step (MFMA decode form): timing at 1/4/16 rows + kernel stats at 16
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 1 4 16; do timeout -k 10 300 python -u scripts/profile_decode.py --batch $b --tokens 512 --prompt 2000 >> gpurun_out/r2_batched_steps.log 2>&1 || exit 1; done
bash scripts/prof_decode.sh r2_dec2k_b16 --batch 16 --tokens 256 --prompt 2000
