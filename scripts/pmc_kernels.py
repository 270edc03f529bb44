"""A few eager launches of each hot kernel, for rocprofv3 --pmc counter collection (counters
serialise dispatches, so no graphs here). Usage on the GPU box:
  cd /tmp && rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \\
      SQ_LDS_IDX_ACTIVE --output-format csv -d <dir> -o run -- python3 scripts/pmc_kernels.py
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from llm_consensus_amd import ops

BF = torch.bfloat16


def main():
    nh, nkv, D, bs = 32, 8, 128, 64
    # flash prefill: 4096 queries over 4096 keys
    T = ctx = 4096
    nb = ctx // bs + 1
    kc = torch.randn(nb, nkv, bs, D, device="cuda").to(BF)
    vc = torch.randn_like(kc)
    bt = torch.arange(nb, dtype=torch.int32, device="cuda").view(1, -1)
    q = torch.randn(T, nh * D, device="cuda").to(BF)
    out = torch.empty_like(q)
    one = lambda v: torch.tensor([v], dtype=torch.int32, device="cuda")  # noqa: E731
    for _ in range(2):
        ops.attn_prefill(q, kc, vc, bt, one(0), one(T), one(ctx), out, T, nh, nkv, D, bs, 1 / math.sqrt(D))
    # decode attention (MFMA split-KV, 32 blocks per kv head) + reduce at 4096 keys
    qd = torch.randn(1, nh * D, device="cuda").to(BF)
    od = torch.empty_like(qd)
    part, ctr = ops.decode_attn_workspace(1, nh, nkv, D, 32, "cuda")
    for _ in range(3):
        ops.attn_decode(qd, kc, vc, bt, one(ctx), od, part, ctr, nh, nkv, D, bs, 128, 1 / math.sqrt(D), grid_chunks=32)
    # decode GEMV: gate_up with fused norm + SiLU epilogue
    W = (torch.randn(28672, 4096, device="cuda") * 0.02).to(BF)
    x = torch.randn(1, 4096, device="cuda").to(BF)
    nw = torch.ones(4096, dtype=BF, device="cuda")
    act = torch.empty(1, 14336, dtype=BF, device="cuda")
    for _ in range(3):
        ops.gemv(x, W, ops.EPI_SILU, out=act, norm_w=nw)
    # our MFMA prefill GEMM (MoE / fallback path)
    xg = torch.randn(2048, 4096, device="cuda").to(BF)
    Wg = (torch.randn(6144, 4096, device="cuda") * 0.02).to(BF)
    for _ in range(2):
        ops.gemm(xg, Wg)
    torch.cuda.synchronize()
    print("pmc driver done")


if __name__ == "__main__":
    main()
