"""Phase timeline of one fused attention + o_proj launch (csrc/kernels/attn_oproj.hip): per-block
s_memrealtime stamps (100 MHz), cold weights (a 1 GiB write flushes the Infinity Cache first).

  python scripts/ao_timeline.py [L ...]
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_consensus_amd import ops  # noqa: E402

BF = torch.bfloat16
NAMES = ["start", "o-attn", "c-attn", "ticket", "head-out", "o-done", "tile-tkt", "reduced"]
NAMES_FR = ["start", "o-attn", "c-attn", "ticket", "heads-in", "o-done", "merged", "published"]  # mode bit 2


def run(L, nh=32, nkv=8, D=128, H=4096, bs=64, mode=0):
    nc = ops.attn_oproj_grid(H, nh, nkv, D)
    cap = 1024
    while cap < L:
        cap *= 2
    chunk = ops.attn_oproj_chunk(cap, nc)
    nb = (L + bs - 1) // bs + 2
    kc = torch.randn(nb, nkv, bs, D, device="cuda").to(BF)
    vc = torch.randn_like(kc)
    bt = torch.randperm(nb, device="cuda")[: (L + bs - 1) // bs].view(1, -1).to(torch.int32)
    sl = torch.full((1,), L, dtype=torch.int32, device="cuda")
    q = torch.randn(1, nh * D, device="cuda").to(BF)
    w_o = (torch.randn(H, nh * D, device="cuda") / math.sqrt(nh * D)).to(BF)
    h = torch.zeros(1, H, dtype=BF, device="cuda")
    attn = torch.zeros(1, nh * D, dtype=BF, device="cuda")
    ws = ops.attn_oproj_workspace(H, nh, nkv, D, nc, "cuda")
    fault = torch.zeros(1, dtype=torch.int32, device="cuda")
    stamps = torch.zeros(nkv, nc, 8, dtype=torch.int64, device="cuda")
    flush = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    for cold in (False, True):
        for _ in range(3):
            ops.attn_oproj(q, kc, vc, bt, sl, w_o, h, attn, ws, nh, nkv, D, bs, chunk, nc, 1 / math.sqrt(D), fault,
                           mode=mode)
        if cold:
            flush.fill_(1)
        stamps.zero_()
        torch.cuda.synchronize()
        ops.attn_oproj(q, kc, vc, bt, sl, w_o, h, attn, ws, nh, nkv, D, bs, chunk, nc, 1 / math.sqrt(D), fault,
                       stamps=stamps, mode=mode)
        torch.cuda.synchronize()
        st = stamps.view(-1, 8).cpu().double()
        t0 = st[:, 0].min()
        print(f"L={L} chunk={chunk} nc={nc} mode={mode} {'cold' if cold else 'warm'} weights: us from the first block's start "
              f"(min / median / max over blocks), fault {int(fault.item())}")
        for k, n in enumerate(NAMES_FR if (mode & 4) and H // nc == 128 and nkv == 8 else NAMES):
            v = st[:, k]
            v = v[v > 0]
            if v.numel() == 0:
                continue
            v = (v - t0) / 100.0
            print(f"  {n:9s} {v.min():7.2f} {v.median():7.2f} {v.max():7.2f}  (n={v.numel()})")


if __name__ == "__main__":
    for L in [int(x) for x in sys.argv[1:]] or [128, 2048]:
        for mode in [int(m) for m in os.environ.get("AO_MODES", "0,1").split(",")]:
            run(L, mode=mode)
