# co-located responders: decode-attention form A/B on a short bench round (scripts/ab_attn_colocated.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A="--results-dir '' --steps 2 --warmup 1 --max-tokens 1024 --warmup-tokens 256"
for i in 1 2; do
  for v in base g8 g4 c256; do
    timeout -k 10 240 bash -c "python scripts/ab_attn_colocated.py $v $A" > gpurun_out/abat_${v}_$i.log 2>&1 || exit 1
  done
done
