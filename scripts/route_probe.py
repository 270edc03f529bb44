"""Microbenchmark of the MoE prefill router (round 6): the router-logits GEMM (M tokens x 8 experts
x K 4096, f32 out) + the top-k kernel against the fused one-launch router, graph-timed on one GPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_consensus_amd import ops  # noqa: E402
from scripts.microbench_kernels import timeit  # noqa: E402

for T in (1024, 2048, 8192):
    x = torch.randn(T, 4096, device="cuda").to(torch.bfloat16)
    wr = (torch.randn(8, 4096, device="cuda") * 0.02).to(torch.bfloat16)
    lg = torch.empty(T, 8, dtype=torch.float32, device="cuda")
    w = torch.empty(T, 2, device="cuda")
    ids = torch.empty(T, 2, dtype=torch.int32, device="cuda")
    g = timeit(lambda: ops.linear(x, wr, ops.EPI_F32, out=lg))
    r = timeit(lambda: ops.moe_route(lg, 2, w, ids))
    f = timeit(lambda: ops.moe_route_fused(x, wr, 2, w, ids))
    print(f"T={T}: router GEMM [{T}x4096]x[8x4096]^T {g:8.2f} us ({ops.gemm_plan(T, 8)}), top-2 {r:8.2f} us; "
          f"fused one-launch router {f:8.2f} us", flush=True)
