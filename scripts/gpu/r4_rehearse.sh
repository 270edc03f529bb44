# Round 4: the 2-, 4- and 8-rank bench flows at full shapes rehearsed on ONE GPU (gloo bootstrap, every
# rank on cuda:0): TP responders / judges with the push-protocol custom collectives and, in the TP
# judges, the one-launch qkv + attention.
cd $GRAFT_REPO_ROOT
tag=${1:-r4reh}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step n2 300 env PORT=29671 bash scripts/rehearse_bench.sh 2 --steps 1 --warmup 1 --max-tokens 256 --judge-max-tokens 16
step n4 300 env PORT=29672 bash scripts/rehearse_bench.sh 4 --steps 1 --warmup 0 --max-tokens 256 --judge-max-tokens 16
step n8 400 env PORT=29673 bash scripts/rehearse_bench.sh 8 --steps 1 --warmup 0 --max-tokens 256 --judge-max-tokens 16
