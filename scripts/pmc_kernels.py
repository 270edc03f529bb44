"""A few eager launches of each hot kernel, for rocprofv3 --pmc counter collection (counters
serialise dispatches, so no graphs here). One counter group per run (scripts/gpu/r2_pmc.sh):
  cd /tmp && rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \\
      SQ_LDS_IDX_ACTIVE --output-format csv -d <dir> -o run -- python3 scripts/pmc_kernels.py

Workloads (Llama-3-8B shapes): flash prefill 4096 x 4096 keys; decode attention in both forms
(fused fixed-chunk at 2k keys, balanced split at 16k keys, merge in the same launch); the decode
GEMVs gate_up (fused norm + SiLU), down (K 14336, residual add) and o_proj (residual add); the
256x256 prefill GEMM on the qkv shape (M 2048) and the gate_up shape (M 4096, SiLU epilogue).
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
    one = lambda v: torch.tensor([v], dtype=torch.int32, device="cuda")  # noqa: E731
    # flash prefill: full causal prompts of PMC_PREFILL tokens (default 4096; "2048,8192": the paired
    # one-round form and the 8-wave multi-round form, both on LDS-DMA staging)
    for T in [int(v) for v in os.environ.get("PMC_PREFILL", "4096").split(",")]:
        ctx = T
        nb = ctx // bs + 1
        kc = torch.randn(nb, nkv, bs, D, device="cuda").to(BF)
        vc = torch.randn_like(kc)
        bt = torch.arange(nb, dtype=torch.int32, device="cuda").view(1, -1)
        q = torch.randn(T, nh * D, device="cuda").to(BF)
        out = torch.empty_like(q)
        for _ in range(2):
            ops.attn_prefill(q, kc, vc, bt, one(0), one(T), one(ctx), out, T, nh, nkv, D, bs, 1 / math.sqrt(D))
        del kc, vc, q, out
    if os.environ.get("PMC_PREFILL_ONLY") == "1":
        torch.cuda.synchronize()
        return

    # decode attention: fused form at 2048 keys (16 chunks of 128), split form at 16384 keys (32
    # 8-wave blocks per kv head); 8 MB and 64 MB of K/V
    qd = torch.randn(1, nh * D, device="cuda").to(BF)
    od = torch.empty_like(qd)
    for L, fused, chunk, gc in ((2048, True, 128, 16), (16384, False, 128, 32)):
        nb = L // bs + 1
        kc = torch.randn(nb, nkv, bs, D, device="cuda").to(BF)
        vc = torch.randn_like(kc)
        bt = torch.arange(nb, dtype=torch.int32, device="cuda").view(1, -1)
        part, ctr = ops.decode_attn_workspace(1, nh, nkv, D, gc, "cuda", fused=fused)
        for _ in range(3):
            ops.attn_decode(qd, kc, vc, bt, one(L), od, part, ctr, nh, nkv, D, bs, chunk, 1 / math.sqrt(D),
                            grid_chunks=gc, fused=fused)
        del kc, vc
    torch.cuda.synchronize()

    # decode GEMVs (weights 235 / 117 / 34 MB)
    x = torch.randn(1, 4096, device="cuda").to(BF)
    nw = torch.ones(4096, dtype=BF, device="cuda")
    Wgu = (torch.randn(28672, 4096, device="cuda") * 0.02).to(BF)
    act = torch.empty(1, 14336, dtype=BF, device="cuda")
    for _ in range(3):
        ops.gemv(x, Wgu, ops.EPI_SILU, out=act, norm_w=nw)
    del Wgu
    Wd = (torch.randn(4096, 14336, device="cuda") * 0.02).to(BF)
    h = torch.zeros(1, 4096, dtype=BF, device="cuda")
    for _ in range(3):
        ops.gemv(act, Wd, ops.EPI_RESADD, out=h)
    del Wd
    Wo = (torch.randn(4096, 4096, device="cuda") * 0.02).to(BF)
    for _ in range(3):
        ops.gemv(x, Wo, ops.EPI_RESADD, out=h)
    del Wo

    # prefill GEMMs
    xg = torch.randn(2048, 4096, device="cuda").to(BF)
    Wg = (torch.randn(6144, 4096, device="cuda") * 0.02).to(BF)
    for _ in range(2):
        ops.gemm(xg, Wg)
    xg = torch.randn(4096, 4096, device="cuda").to(BF)
    Wg = (torch.randn(28672, 4096, device="cuda") * 0.02).to(BF)
    for _ in range(2):
        ops.gemm(xg, Wg, ops.EPI_SILU)
    torch.cuda.synchronize()
    print("pmc driver done")


if __name__ == "__main__":
    main()
