set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/profile_decode.py --prompt 32500 --ctx 33300 --tokens 256 > gpurun_out/r2_ref_8b_33k.log 2>&1 && \
timeout -k 10 300 python scripts/profile_decode.py --prompt 2048 --ctx 8192 --tokens 512 > gpurun_out/r2_ref_8b_2k.log 2>&1 && \
timeout -k 10 300 python scripts/profile_decode.py --model mixtral-8x7b --prompt 2048 --ctx 8192 --tokens 256 > gpurun_out/r2_ref_mixtral.log 2>&1 && \
timeout -k 10 300 python scripts/profile_decode.py --model phi-3-mini --prompt 2048 --ctx 8192 --tokens 512 > gpurun_out/r2_ref_phi3.log 2>&1 && \
timeout -k 10 400 python scripts/profile_decode.py --model llama-3-70b --prompt 2048 --ctx 4096 --tokens 64 > gpurun_out/r2_ref_70b.log 2>&1
