"""Run the prefill GEMM and hipBLASLt back to back on one shape (for rocprofv3 --pmc passes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from llm_consensus_amd import ops

M, N, K = 8192, 28672, 4096
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
W = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
for _ in range(5):
    ops.gemm(x, W, 0, out=out)
    torch.matmul(x, W.t(), out=out)
torch.cuda.synchronize()
print("done")
