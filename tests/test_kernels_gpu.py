"""Kernel numerics on a real MI355X: each HIP kernel vs the fp32 PyTorch oracle of the same op
(SURVEY.md §4.2 "Kernel numerics")."""

import math

import pytest
import torch

from llm_consensus_amd import ops
from llm_consensus_amd.ops import oracle

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def rnd(*shape, scale=1.0, dev="cuda"):
    return (torch.randn(*shape, device=dev) * scale).to(BF)


def close(a, b, atol, rtol=0.02):
    a = a.float().cpu()
    b = b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{bad}/{a.numel()} mismatches, max err {err.max().item():.4g}"


def _normed_exact(x, nw, eps=1e-5):
    """fp32 rmsnorm(x) * w, unrounded: the exact input of a fused-norm projection."""
    xf = x.cpu().float()
    return xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * nw.cpu().float()


def test_lane_exchange_helpers_match_shfl_xor(cuda):
    """The kernels' wave reductions and lane exchanges (v_permlane16/32_swap, DPP row_ror / quad_perm
    / bank-masked rotations in csrc/kernels/common.h) against the ds_bpermute (__shfl_xor) forms they
    replace: the same association order, so every pair is bit-identical — including the +-0 and
    equal-magnitude cases the random data hits."""
    torch.manual_seed(5)
    x = torch.randn(64 * 64, device="cuda") * 50
    x[:2048:2] = -x[1:2048:2]  # exact cancellations in the first 32 waves
    x[3::11] = 0.0
    got = ops.lane_exchange_check(x).cpu()
    a, b = got[..., 0], got[..., 1]
    bad = (a.view(torch.int32) != b.view(torch.int32)).nonzero()
    assert bad.numel() == 0, f"{bad.shape[0]} mismatches, first (lane, check): {bad[:5].tolist()}"


def no_worse_than_oracle(got, ref, exact, slack=1e-2):
    """The MFMA decode form (3-16 rows) factorises the fused norm — bf16(x * w), scaled by 1/rms
    in f32 — where the oracle rounds bf16(x / rms * w): each is one bf16 rounding away from the
    exact math. Pass when the kernel is no further from the exact result than the oracle."""
    e_k = (got.float().cpu() - exact.float()).abs().max().item()
    e_o = (ref.float().cpu() - exact.float()).abs().max().item()
    assert e_k <= 1.5 * e_o + slack, (e_k, e_o)


@pytest.mark.parametrize("H", [256, 3072, 4096, 8192])
def test_rmsnorm(cuda, H):
    torch.manual_seed(0)
    x = rnd(7, H)
    w = rnd(H)
    y = ops.rmsnorm(x, w, 1e-5)
    close(y, oracle.rmsnorm(x.cpu(), w.cpu(), 1e-5), 1e-2)


def test_embedding_and_silu(cuda):
    torch.manual_seed(0)
    tab = rnd(1000, 512)
    ids = torch.tensor([0, 5, 999, 17], dtype=torch.int32, device="cuda")
    assert torch.equal(ops.embedding(ids, tab).cpu(), oracle.embedding(ids.cpu(), tab.cpu()))
    gu = rnd(9, 2 * 768)
    close(ops.silu_mul_interleaved(gu), oracle.silu_mul_interleaved(gu.cpu()), 1e-2)


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,K", [(64, 256), (1000, 4096), (4096, 4096), (512, 14336), (130, 192), (6144, 512), (9216, 256),
                                 (1792, 4096), (4096, 14336)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_gemv(cuda, M, N, K, epi):
    """Every decode row count (replica / continuous batching: M = 2-4) on every shape class,
    including the 8B down_proj (K = 14336: x rows staged in up to 112 KiB of LDS)."""
    torch.manual_seed(M * 7 + N + K + epi)
    x = rnd(M, K)
    W = rnd(N, K, scale=0.05)
    out = rnd(M, N) if epi == 2 else None
    ref_out = out.cpu().clone() if out is not None else None
    y = ops.gemv(x, W, epi, out=out)
    ref = oracle.linear(x.cpu(), W.cpu(), epi, ref_out)
    close(y, ref, 2e-2)


@pytest.mark.parametrize("M", [1, 2, 3, 4])
def test_gemv_fused_norm(cuda, M):
    torch.manual_seed(1)
    x = rnd(M, 4096)
    W = rnd(6144, 4096, scale=0.05)
    nw = rnd(4096)
    y = ops.gemv(x, W, 0, norm_w=nw, eps=1e-5)
    ref = oracle.linear(x.cpu(), W.cpu(), 0, None, nw.cpu(), 1e-5)
    if M <= 2:
        close(y, ref, 3e-2)
    else:
        no_worse_than_oracle(y, ref, _normed_exact(x, nw) @ W.cpu().float().t())


@pytest.mark.parametrize("M", [1, 4, 5, 8, 16, 17, 24, 32])
@pytest.mark.parametrize("N,K", [(64, 256), (1000, 4096), (136, 384), (6144, 512), (4096, 14336), (28672, 4096)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_gemvm(cuda, M, N, K, epi):
    """The MFMA weight-streaming form (batched decode, gemv_mfma.hip) on its own, every epilogue:
    split-K over 1-16 waves (K 256 -> 2 waves of one 128-k tile, 14336 -> 8 waves), ragged N
    (clamped rows, masked stores), tokens M < 16 (clamped x rows, discarded columns), 17-32 tokens
    (two 16-token column groups per weight fragment)."""
    torch.manual_seed(M * 5 + N + K + epi)
    x = rnd(M, K)
    W = rnd(N, K, scale=0.05)
    out = rnd(M, N) if epi == 2 else None
    ref_out = out.cpu().clone() if out is not None else None
    y = ops.gemvm(x, W, epi, out=out)
    ref = oracle.linear(x.cpu(), W.cpu(), epi, ref_out)
    close(y, ref, 2e-2)


@pytest.mark.parametrize("B", [3, 8, 16])
@pytest.mark.parametrize("ep", [False, True])
def test_moe_gemvm(cuda, B, ep):
    """Batched MoE decode with the (token, slot) pairs grouped by expert (MFMA form): gate_up with
    the fused norm + SiLU and the down projection, per pair against the fp32 oracle; expert-parallel
    ids (-1 = another rank's expert) leave their rows untouched."""
    torch.manual_seed(B * 3 + ep)
    E, H, I, k = 8, 512, 384, 2
    ids = torch.stack([torch.randperm(E)[:k] for _ in range(B)]).to(torch.int32)
    if ep:
        ids[ids >= 4] = -1
    x = rnd(B, H)
    nw = rnd(H)
    Wgu = rnd(E, 2 * I, H, scale=0.05)
    Wd = rnd(E, H, I, scale=0.05)
    act = torch.full((B * k, I), 7.0, dtype=BF, device="cuda")
    y = torch.full((B * k, H), 7.0, dtype=BF, device="cuda")
    ops.moe_gemvm(x, Wgu, ids.cuda(), k, act, 2 * I, H, ops.EPI_SILU, norm_w=nw, eps=1e-5)
    ops.moe_gemvm(act, Wd, ids.cuda(), 1, y, H, I, ops.EPI_BF16)
    xn = _normed_exact(x, nw)
    for p, e in enumerate(ids.view(-1).tolist()):
        if e < 0:
            assert bool((act[p] == 7.0).all()) and bool((y[p] == 7.0).all()), p
            continue
        ref = oracle.linear(x[p // k:p // k + 1].cpu(), Wgu[e].cpu(), ops.EPI_SILU, None, nw.cpu(), 1e-5)
        g = xn[p // k:p // k + 1] @ Wgu[e].cpu().float().t()
        no_worse_than_oracle(act[p:p + 1], ref, torch.nn.functional.silu(g[:, 0::2]) * g[:, 1::2])
        close(y[p:p + 1], oracle.linear(act[p:p + 1].cpu(), Wd[e].cpu(), ops.EPI_BF16), 2e-2)


@pytest.mark.parametrize("form", [1, 2, 3, 4])
@pytest.mark.parametrize("M", [3, 16, 29])
@pytest.mark.parametrize("N,K", [(1000, 4096), (8200, 1024), (4096, 14336)])
@pytest.mark.parametrize("epi", [0, 2, 3])
def test_gemvm_forms(cuda, form, M, N, K, epi):
    """Every variant of the MFMA form pinned (one / two 16-row weight groups per wave, x fragments
    from L2 / through LDS): ragged N for the 32-row blocks (1000, 8200), split-K 4-8 waves."""
    torch.manual_seed(form * 13 + M + N + epi)
    x = rnd(M, K)
    W = rnd(N, K, scale=0.05)
    out = rnd(M, N) if epi == 2 else None
    ref_out = out.cpu().clone() if out is not None else None
    if M > 16 and form == 4:  # two x tiles per token group beside two weight groups: over the LDS
        with pytest.raises(RuntimeError):
            ops.gemvm(x, W, epi, out=out, form=form)
        return
    y = ops.gemvm(x, W, epi, out=out, form=form)
    close(y, oracle.linear(x.cpu(), W.cpu(), epi, ref_out), 2e-2)


@pytest.mark.parametrize("M", [3, 5, 7, 12, 16, 20, 32])
@pytest.mark.parametrize("N,K,epi", [(6144, 4096, 0), (28672, 4096, 3), (4096, 14336, 2), (128256, 4096, 1),
                                     (9216, 3072, 0)])
def test_linear_batched_decode_rows(cuda, M, N, K, epi):
    """ops.linear at continuous-batching row counts (3-32) on the Llama-3-8B / Phi-3 decode shapes:
    the dispatcher must take the MFMA form (fused norm prologue where the layer has one)."""
    torch.manual_seed(M + N + epi)
    x = rnd(M, K)
    W = rnd(N, K, scale=0.05)
    nw = rnd(K) if epi in (0, 1, 3) else None
    out = rnd(M, N) if epi == 2 else None
    ref_out = out.cpu().clone() if out is not None else None
    y = ops.linear(x, W, epi, out=out, norm_w=nw, eps=1e-5)
    ref = oracle.linear(x.cpu(), W.cpu(), epi, ref_out.clone() if ref_out is not None else None,
                        nw.cpu() if nw is not None else None, 1e-5)
    if nw is None:
        close(y, ref, 3e-2)
        return
    acc = _normed_exact(x, nw) @ W.cpu().float().t()
    no_worse_than_oracle(y, ref, {0: acc, 1: acc, 3: torch.nn.functional.silu(acc[:, 0::2]) * acc[:, 1::2]}[epi])


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (37, 200, 256), (300, 512, 4096), (1024, 384, 1024),
                                   (5, 4096, 128), (600, 700, 1472), (257, 130, 320), (2048, 2304, 2048),
                                   (513, 6144, 4096)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_gemm(cuda, M, N, K, epi):
    """256x256 ring-pipelined prefill GEMM vs the fp32 oracle: ragged M/N tiles (row/column
    clamps, masked epilogue), N % 4 != 0 (scalar epilogue), K from one to 64 K-steps (ring
    wrap-around, the vmcnt(0) tail), every epilogue incl. the fused SiLU-mul."""
    if epi == 3 and N % 2:
        pytest.skip("SiLU pairs need even N")
    torch.manual_seed(M + N + K + epi)
    x = rnd(M, K)
    W = rnd(N, K, scale=0.05)
    out = rnd(M, N) if epi == 2 else None
    ref_out = out.cpu().clone() if out is not None else None
    y = ops.gemm256(x, W, epi, out=out)
    ref = oracle.linear(x.cpu(), W.cpu(), epi, ref_out)
    close(y, ref, 2e-2)


@pytest.mark.parametrize("M,N,K", [(8192, 768, 512), (4100, 1536, 256), (4096, 4096, 128)])
def test_gemm_dispatch(cuda, M, N, K):
    """ops.gemm through llmc_gemm's kernel choice on shapes either side of the narrow-N rule
    (gemm_plan: 128 x 192 for 8192 x 768, 256 x 256 for 4096 x 4096) vs the fp32 oracle."""
    torch.manual_seed(M + N + K)
    x = rnd(M, K)
    W = rnd(N, K, scale=0.05)
    close(ops.gemm(x, W, 0), oracle.linear(x.cpu(), W.cpu(), 0, None), 2e-2)


@pytest.mark.parametrize("M,N,K", [(300, 768, 4096), (1024, 2560, 1024), (257, 130, 320), (37, 200, 256)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_gemm128_dense(cuda, M, N, K, epi):
    """The 128 x 128 two-buffer kernel on dense problems (the narrow-N prefill dispatch: a TP rank's
    qkv / o shards) vs the fp32 oracle, every epilogue, ragged tiles."""
    if epi == 3 and N % 2:
        pytest.skip("SiLU pairs need even N")
    torch.manual_seed(M + N + K + epi + 7)
    x = rnd(M, K)
    W = rnd(N, K, scale=0.05)
    out = rnd(M, N) if epi == 2 else None
    ref_out = out.cpu().clone() if out is not None else None
    y = ops.gemm128(x, W, epi, out=out)
    ref = oracle.linear(x.cpu(), W.cpu(), epi, ref_out)
    close(y, ref, 2e-2)


@pytest.mark.parametrize("M,N,K", [(300, 768, 4096), (1024, 2560, 1024), (257, 130, 320), (37, 200, 256),
                                   (128, 192, 64), (200, 384, 128), (129, 194, 192)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_gemm_narrow(cuda, M, N, K, epi):
    """The 128 x 192 narrow-N kernel vs the fp32 oracle: every epilogue, ragged M / N tiles, K of one,
    two and three K-steps (the prologue's vmcnt forms) up to 64 (the 3-slot ring wrapping)."""
    if epi == 3 and N % 2:
        pytest.skip("SiLU pairs need even N")
    torch.manual_seed(M + N + K + epi + 11)
    x = rnd(M, K)
    W = rnd(N, K, scale=0.05)
    out = rnd(M, N) if epi == 2 else None
    ref_out = out.cpu().clone() if out is not None else None
    y = ops.gemm_narrow(x, W, epi, out=out)
    ref = oracle.linear(x.cpu(), W.cpu(), epi, ref_out)
    close(y, ref, 2e-2)


@pytest.mark.parametrize("K", [128, 512])
def test_gemm_narrow_identity_asymmetric(cuda, K):
    """A = I against an asymmetric W through the narrow kernel: a transposed or misplaced C write
    shows as a wrong element (K = 512: 4 M tiles x 3 N tiles, the last one partial)."""
    A = torch.eye(K, dtype=BF, device="cuda")
    W = (torch.arange(K * K, device="cuda").view(K, K) % 97).to(BF)
    assert torch.equal(ops.gemm_narrow(A, W, 0).cpu(), W.t().contiguous().cpu())


@pytest.mark.parametrize("K", [128, 512])
def test_gemm_identity_asymmetric(cuda, K):
    """A = I with an asymmetric B catches a transposed C write (guide §3); K = 512 spans two
    256-row tiles in M and N."""
    A = torch.eye(K, dtype=BF, device="cuda")
    W = (torch.arange(K * K, device="cuda").view(K, K) % 97).to(BF)  # asymmetric
    y = ops.gemm256(A, W, 0)
    assert torch.equal(y.cpu(), W.t().contiguous().cpu())


def _rope_setup(nh, nkv, D, T, bs=64, nblocks=8):
    from llm_consensus_amd.models.config import LLAMA3_8B, rope_inv_freq

    cos_t, sin_t = oracle.rope_tables(rope_inv_freq(LLAMA3_8B.with_(head_dim=D)), 4096)
    qkv = rnd(T, (nh + 2 * nkv) * D)
    pos = torch.randint(0, 4000, (T,), dtype=torch.int32)
    perm = torch.randperm(nblocks * bs)[:T].to(torch.int32)
    kc = torch.zeros(nblocks, nkv, bs, D, dtype=BF)
    vc = torch.zeros_like(kc)
    return cos_t, sin_t, qkv, pos, perm, kc, vc


@pytest.mark.parametrize("nh,nkv,D", [(32, 8, 128), (32, 32, 96), (4, 2, 64)])
def test_rope_kv_write(cuda, nh, nkv, D):
    torch.manual_seed(2)
    cos_t, sin_t, qkv, pos, slots, kc, vc = _rope_setup(nh, nkv, D, 11)
    kc_ref, vc_ref = kc.clone(), vc.clone()
    q_ref = torch.zeros(11, nh * D, dtype=BF)
    oracle.rope_kv_write(qkv.cpu(), pos, cos_t, sin_t, kc_ref, vc_ref, slots, nh, nkv, D, 64, q_ref)
    kd, vd = kc.cuda(), vc.cuda()
    qd = torch.zeros(11, nh * D, dtype=BF, device="cuda")
    ops.rope_kv_write(qkv, pos.cuda(), cos_t.cuda(), sin_t.cuda(), kd, vd, slots.cuda(), nh, nkv, D, 64, qd)
    close(qd, q_ref, 1e-2)
    close(kd, kc_ref, 1e-2)
    assert torch.equal(vd.cpu(), vc_ref)


@pytest.mark.parametrize("M", [1, 2, 3, 4, 5, 8, 16, 19, 32])
@pytest.mark.parametrize("nh,nkv,D,H", [(32, 8, 128, 4096), (32, 32, 96, 3072), (4, 2, 64, 256), (16, 2, 128, 8192),
                                          (4, 1, 128, 4096), (8, 2, 128, 4096)])
def test_gemv_qkv_rope(cuda, M, nh, nkv, D, H):
    """Fused decode qkv GEMV (norm prologue + RoPE/KV-write epilogue) vs the 2-step oracle."""
    torch.manual_seed(12)
    cos_t, sin_t, _, pos, slots, kc, vc = _rope_setup(nh, nkv, D, M)
    N = (nh + 2 * nkv) * D
    x = rnd(M, H)
    W = rnd(N, H, scale=0.05)
    nw = rnd(H)
    kc_ref, vc_ref = kc.clone(), vc.clone()
    q_ref = torch.zeros(M, nh * D, dtype=BF)
    qkv = oracle.linear(x.cpu(), W.cpu(), 0, None, nw.cpu(), 1e-5)
    oracle.rope_kv_write(qkv, pos, cos_t, sin_t, kc_ref, vc_ref, slots, nh, nkv, D, 64, q_ref)
    kd, vd = kc.cuda(), vc.cuda()
    qd = torch.zeros(M, nh * D, dtype=BF, device="cuda")
    ops.qkv_rope(x, W, nw, 1e-5, qd, kd, vd, pos.cuda(), slots.cuda(), cos_t.cuda(), sin_t.cuda(), nh, nkv, D, 64)
    if M <= 2:
        close(qd, q_ref, 3e-2)
        close(kd, kc_ref, 3e-2)
        close(vd, vc_ref, 3e-2)
        return
    # 3-16 rows (MFMA form, factorised norm): against the exact fp32 math, next to the oracle
    kc_x, vc_x = kc.clone(), vc.clone()
    q_x = torch.zeros(M, nh * D, dtype=BF)
    oracle.rope_kv_write(_normed_exact(x, nw) @ W.cpu().float().t(), pos, cos_t, sin_t, kc_x, vc_x, slots, nh, nkv, D,
                         64, q_x)
    for got, ref, ex in ((qd, q_ref, q_x), (kd, kc_ref, kc_x), (vd, vc_ref, vc_x)):
        no_worse_than_oracle(got, ref, ex)


def _paged_kv(B, L_max, nkv, D, bs):
    nblk_per = (L_max + bs - 1) // bs
    nb = B * nblk_per + 3
    kc = rnd(nb, nkv, bs, D)
    vc = rnd(nb, nkv, bs, D)
    perm = torch.randperm(nb)[: B * nblk_per].view(B, nblk_per).to(torch.int32)
    return kc, vc, perm


@pytest.mark.parametrize("nh,nkv,D", [(32, 8, 128), (32, 32, 96), (16, 2, 128), (4, 2, 64), (64, 8, 128), (8, 1, 128)])
@pytest.mark.parametrize("lens", [[1, 7], [100, 1000], [3000, 257], [4096, 128, 129, 2049]])
@pytest.mark.parametrize("chunk", [128, 256])
def test_attn_decode_fused(cuda, nh, nkv, D, lens, chunk):
    """Short-context form: fixed 128/256-key chunks (a 4096-key bucket = 32/16 blocks per kv head),
    merged in the same launch by the last-arriving block from tagged granules; the ticket must be
    re-armed and the epoch of every (row, kv head) that merged advanced once per launch."""
    torch.manual_seed(3)
    B, bs = len(lens), 64
    kc, vc, bt = _paged_kv(B, max(lens), nkv, D, bs)
    q = rnd(B, nh * D)
    sl = torch.tensor(lens, dtype=torch.int32)
    gc = 4096 // chunk
    part, ctr = ops.decode_attn_workspace(B, nh, nkv, D, gc, "cuda", fused=True)
    out = torch.empty(B, nh * D, dtype=BF, device="cuda")
    scale = 1 / math.sqrt(D)
    ref = oracle.attn_decode(q.cpu(), kc.cpu(), vc.cpu(), bt, sl, nh, nkv, D, bs, scale)
    for _ in range(3):
        out.zero_()
        ops.attn_decode(q, kc, vc, bt.cuda(), sl.cuda(), out, part, ctr, nh, nkv, D, bs, chunk, scale, grid_chunks=gc,
                        fused=True)
        close(out, ref, 2e-2)
    # tickets re-armed, epochs advanced once per launch where a merge ran
    epochs = torch.tensor([3 if n > chunk else 0 for n in lens], dtype=torch.int32).view(-1, 1).expand(B, nkv)
    assert int(ctr[..., 0, 0].abs().sum()) == 0 and torch.equal(ctr[..., 1, 0].cpu(), epochs), ctr
    assert int(ctr[..., 1:].abs().sum()) == 0  # one word per 128-B counter line


@pytest.mark.parametrize("nh,nkv,D", [(32, 8, 128), (32, 32, 96), (16, 2, 128)])
@pytest.mark.parametrize("gc", [1, 3, 7, 64])
def test_attn_decode_balanced_split(cuda, nh, nkv, D, gc):
    """Long-context form with a fixed grid: each sequence's keys spread evenly over gc 8-wave blocks
    (>= 128 keys each), merged in the same launch. The lengths change between launches on the same
    workspace (a row's chunk count shrinks and grows back), so a granule left by an earlier launch
    must never be taken for this one's."""
    torch.manual_seed(5)
    bs = 64
    rounds = [[5000, 130, 1], [5000, 130, 1], [300, 4999, 2], [4097, 3000, 700], [5000, 130, 1]]
    B = 3
    kc, vc, bt = _paged_kv(B, 5000, nkv, D, bs)
    q = rnd(B, nh * D)
    part, ctr = ops.decode_attn_workspace(B, nh, nkv, D, gc, "cuda")
    out = torch.empty(B, nh * D, dtype=BF, device="cuda")
    scale = 1 / math.sqrt(D)
    for lens in rounds:
        sl = torch.tensor(lens, dtype=torch.int32)
        ref = oracle.attn_decode(q.cpu(), kc.cpu(), vc.cpu(), bt, sl, nh, nkv, D, bs, scale)
        out.zero_()
        ops.attn_decode(q, kc, vc, bt.cuda(), sl.cuda(), out, part, ctr, nh, nkv, D, bs, 128, scale, grid_chunks=gc)
        close(out, ref, 2e-2)


@pytest.mark.parametrize("nh,nkv,chunk,cap", [(4, 1, 128, 32768), (4, 1, 256, 65536), (16, 2, 256, 32768)])
def test_attn_decode_fused_long_context(cuda, nh, nkv, chunk, cap):
    """The fixed-chunk form on TP ranks at judge lengths (engine.attn_buckets: one or two kv heads
    over up to 256 chunk blocks, merged in two levels of 16), lengths changing between launches on
    one workspace."""
    torch.manual_seed(8)
    D, bs, B = 128, 64, 3
    Lmax = min(cap, 40000)
    kc, vc, bt = _paged_kv(B, Lmax, nkv, D, bs)
    q = rnd(B, nh * D)
    gc = cap // chunk
    part, ctr = ops.decode_attn_workspace(B, nh, nkv, D, gc, "cuda", fused=True)
    out = torch.empty(B, nh * D, dtype=BF, device="cuda")
    scale = 1 / math.sqrt(D)
    for lens in ([Lmax, 9000, 130], [2100, Lmax - 1, 17000], [Lmax, 9000, 130]):
        sl = torch.tensor(lens, dtype=torch.int32)
        ref = oracle.attn_decode(q.cpu(), kc.cpu(), vc.cpu(), bt, sl, nh, nkv, D, bs, scale)
        out.zero_()
        ops.attn_decode(q, kc, vc, bt.cuda(), sl.cuda(), out, part, ctr, nh, nkv, D, bs, chunk, scale,
                        grid_chunks=gc, fused=True)
        close(out, ref, 2e-2)
    tickets = torch.cat([ctr[..., :1, 0], ctr[..., 2:, 0]], dim=-1)
    assert int(tickets.abs().sum()) == 0, ctr


@pytest.mark.parametrize("nh,nkv", [(4, 1), (8, 1), (16, 2)])
@pytest.mark.parametrize("gc", [100, 256, 300])
def test_attn_decode_wide_split(cuda, nh, nkv, gc):
    """TP ranks at judge-length contexts (a TP=8 rank of Llama-3-8B: 4 query heads on ONE kv head;
    Llama-3-70B TP=8 / TP=4 ranks: G = 8): the keys spread over up to 300 blocks, so the partials
    merge in two levels (groups of 16, then the group results). Lengths change between launches on
    the same workspace; every ticket must be re-armed."""
    torch.manual_seed(6)
    D, bs = 128, 64
    B = 3
    kc, vc, bt = _paged_kv(B, 40000, nkv, D, bs)
    q = rnd(B, nh * D)
    part, ctr = ops.decode_attn_workspace(B, nh, nkv, D, gc, "cuda")
    out = torch.empty(B, nh * D, dtype=BF, device="cuda")
    scale = 1 / math.sqrt(D)
    for lens in ([40000, 9000, 130], [2100, 39999, 17000], [40000, 9000, 130]):
        sl = torch.tensor(lens, dtype=torch.int32)
        ref = oracle.attn_decode(q.cpu(), kc.cpu(), vc.cpu(), bt, sl, nh, nkv, D, bs, scale)
        out.zero_()
        ops.attn_decode(q, kc, vc, bt.cuda(), sl.cuda(), out, part, ctr, nh, nkv, D, bs, 128, scale, grid_chunks=gc)
        close(out, ref, 2e-2)
    tickets = torch.cat([ctr[..., :1, 0], ctr[..., 2:, 0]], dim=-1)
    assert int(tickets.abs().sum()) == 0, ctr


def test_attn_decode_partial_rounding_at_33k(cuda):
    """each chunk's normalised partial O/l is published in bf16, and the two-level merge
    (256 blocks = 16 groups of 16) rounds the group results to bf16 again. Measured against an fp32
    attention at 33k keys on a TP=8 rank's shape (4 query heads on one kv head): the error of the
    256-block two-level path vs that of ONE block (no published partials: f32 wave merge, one
    bf16 rounding of the output). The extra roundings must stay within bf16's own rounding of the
    output (recorded in the assertion message)."""
    torch.manual_seed(12)
    nh, nkv, D, bs, L = 4, 1, 128, 64, 33000
    kc, vc, bt = _paged_kv(1, L, nkv, D, bs)
    q = rnd(1, nh * D)
    sl = torch.tensor([L], dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    # fp32 reference on the GPU
    idx = torch.arange(L, device="cuda")
    pages = bt[0].cuda().long()[idx // bs]
    k = kc[pages, 0, idx % bs].float()
    v = vc[pages, 0, idx % bs].float()
    p = torch.softmax((q.view(nh, D).float() @ k.t()) * scale, dim=-1)
    ref = (p @ v).view(1, -1)
    errs = {}
    for gc in (1, 256):
        part, ctr = ops.decode_attn_workspace(1, nh, nkv, D, gc, "cuda")
        out = torch.zeros(1, nh * D, dtype=BF, device="cuda")
        ops.attn_decode(q, kc, vc, bt.cuda(), sl.cuda(), out, part, ctr, nh, nkv, D, bs, 128, scale, grid_chunks=gc)
        torch.cuda.synchronize()
        errs[gc] = (out.float() - ref).abs().max().item()
    bf16_ulp = ref.abs().max().item() * 2 ** -8
    assert errs[256] <= errs[1] + bf16_ulp, (errs, bf16_ulp)


@pytest.mark.parametrize("ksplit", [1, 2, 4])
@pytest.mark.parametrize("nh,nkv,D", [(32, 8, 128), (32, 32, 96), (16, 2, 128), (4, 2, 64)])
@pytest.mark.parametrize("case", ["full", "chunk", "ragged"])
def test_attn_prefill(cuda, nh, nkv, D, case, ksplit):
    """ksplit > 1: each row-tile group's key tiles split over that many blocks + the merge launch
    (ragged: 1-key contexts leave most splits empty)."""
    torch.manual_seed(4)
    bs = 64
    if case == "full":
        qlens, ctx = [300], [300]
    elif case == "chunk":
        qlens, ctx = [200, 64], [1000, 64]
    else:
        qlens, ctx = [1, 33, 130], [1, 97, 700]
    B = len(qlens)
    kc, vc, bt = _paged_kv(B, max(ctx), nkv, D, bs)
    qs = torch.tensor([0] + list(torch.cumsum(torch.tensor(qlens), 0)[:-1]), dtype=torch.int32)
    T = sum(qlens)
    q = rnd(T, nh * D)
    out = torch.zeros(T, nh * D, dtype=BF, device="cuda")
    ql = torch.tensor(qlens, dtype=torch.int32)
    cl = torch.tensor(ctx, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    ops.attn_prefill(q, kc, vc, bt.cuda(), qs.cuda(), ql.cuda(), cl.cuda(), out, max(qlens), nh, nkv, D, bs, scale,
                     max_ctx=max(ctx), ksplit=ksplit, kmin=1)
    ref = torch.zeros(T, nh * D, dtype=BF)
    oracle.attn_prefill(q.cpu(), kc.cpu(), vc.cpu(), bt, qs, ql, cl, nh, nkv, D, bs, scale, ref)
    close(out, ref, 2e-2)


def test_attn_prefill_split_is_deterministic_and_leaves_foreign_rows(cuda):
    """A split launch (the last split block to arrive merges) gives the same bits on every run
    whichever block arrives last, matches the unsplit kernel to bf16 rounding, and leaves rows
    outside every sequence's [q_start, q_start + q_len) untouched, as the unsplit kernel does."""
    torch.manual_seed(9)
    nh, nkv, D, bs = 8, 2, 128, 64
    qlens, ctx = [100, 50], [1600, 50]
    kc, vc, bt = _paged_kv(2, max(ctx), nkv, D, bs)
    qs = torch.tensor([0, 110], dtype=torch.int32)  # rows 100..109 and 160..169 belong to no sequence
    T = 170
    q = rnd(T, nh * D)
    ql, cl = torch.tensor(qlens, dtype=torch.int32), torch.tensor(ctx, dtype=torch.int32)
    ws = ops.attn_prefill_workspace(4, T, nh, D, "cuda", 2, nkv, max(qlens))
    outs = []
    for k in (1, 4, 4, 4):
        out = torch.full((T, nh * D), 7.0, dtype=BF, device="cuda")
        ops.attn_prefill(q, kc, vc, bt.cuda(), qs.cuda(), ql.cuda(), cl.cuda(), out, max(qlens), nh, nkv, D, bs,
                         1 / math.sqrt(D), max_ctx=max(ctx), ksplit=k, kmin=2, ws=ws)
        outs.append(out)
    torch.cuda.synchronize()
    for out in outs:
        assert (out[100:110] == 7.0).all() and (out[160:] == 7.0).all()
    assert torch.equal(outs[1], outs[2]) and torch.equal(outs[1], outs[3])
    assert (ws[1] == 0).all()  # counters re-armed for the next layer
    close(outs[1], outs[0].float().cpu(), 2e-2)


@pytest.mark.parametrize("nh,nkv,D,ctx", [(32, 8, 128, 8192), (32, 8, 128, 16384), (32, 8, 128, 33000),
                                        (32, 32, 96, 16384)])
@pytest.mark.parametrize("ksplit", [1, 4])
def test_attn_prefill_long_context_vs_fp32(cuda, nh, nkv, D, ctx, ksplit):
    """Judge-length contexts (the N=8 judge prompt is ~33k tokens): the last 384 queries of a ctx-key
    paged sequence (the final chunk of a chunked prefill) beside a short full prefill, against the
    fp32 oracle computed on the GPU (the same einsum/softmax code as the CPU oracle)."""
    torch.manual_seed(ctx + D)
    bs = 64
    qlens, ctxs = [384, 300], [ctx, 300]
    B = len(qlens)
    kc, vc, bt = _paged_kv(B, max(ctxs), nkv, D, bs)
    qs = torch.tensor([0, qlens[0]], dtype=torch.int32)
    T = sum(qlens)
    q = rnd(T, nh * D)
    out = torch.zeros(T, nh * D, dtype=BF, device="cuda")
    ql, cl = torch.tensor(qlens, dtype=torch.int32), torch.tensor(ctxs, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    ops.attn_prefill(q, kc, vc, bt.cuda(), qs.cuda(), ql.cuda(), cl.cuda(), out, max(qlens), nh, nkv, D, bs, scale,
                     max_ctx=max(ctxs), ksplit=ksplit, kmin=4)
    ref = torch.zeros(T, nh * D, dtype=BF, device="cuda")
    oracle.attn_prefill(q, kc, vc, bt.cuda(), qs, ql, cl, nh, nkv, D, bs, scale, ref)  # fp32 math, on the GPU
    torch.cuda.synchronize()
    close(out, ref.float().cpu(), 2e-2)


@pytest.mark.parametrize("nh,nkv,D,qlens", [(32, 8, 128, [2048]), (32, 8, 128, [1000, 700]), (32, 32, 96, [1024]),
                                          (16, 2, 128, [1500]), (8, 1, 128, [640, 130])])
@pytest.mark.parametrize("form", [0, 1, 2, 3])
def test_attn_prefill_block_forms_vs_fp32(cuda, nh, nkv, D, qlens, form):
    """Every block form of the unsplit prefill forced on the same problems against the fp32 oracle:
    8-wave blocks (LDS-DMA staging for D = 128 on 64-key pages, register staging for D = 96), paired
    late / early row tiles (G <= 4; G = 8 falls back to 8 waves), 4-wave blocks and key halves (two
    wave halves over the two halves of the key tiles, merged through LDS; D = 128 only, else 8
    waves); full and ragged sequences, a short second sequence beside a long one."""
    torch.manual_seed(sum(qlens) + D + form)
    bs = 64
    B = len(qlens)
    kc, vc, bt = _paged_kv(B, max(qlens), nkv, D, bs)
    qs = torch.tensor([sum(qlens[:i]) for i in range(B)], dtype=torch.int32)
    T = sum(qlens)
    q = rnd(T, nh * D)
    out = torch.zeros(T, nh * D, dtype=BF, device="cuda")
    ql = torch.tensor(qlens, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    ops.attn_prefill(q, kc, vc, bt.cuda(), qs.cuda(), ql.cuda(), ql.cuda(), out, max(qlens), nh, nkv, D, bs, scale,
                     ksplit=1, form=form)
    ref = torch.zeros(T, nh * D, dtype=BF, device="cuda")
    oracle.attn_prefill(q, kc, vc, bt.cuda(), qs, ql, ql, nh, nkv, D, bs, scale, ref)
    torch.cuda.synchronize()
    close(out, ref.float().cpu(), 2e-2)


def _sample_bufs(B, V):
    P = ops.sample_parts()
    return (torch.empty(B, P, device="cuda"), torch.empty(B, P, dtype=torch.int32, device="cuda"),
            torch.empty(B, dtype=torch.int32, device="cuda"))


@pytest.mark.parametrize("V", [1000, 128256])
def test_sample_greedy_and_gumbel(cuda, V):
    torch.manual_seed(5)
    B = 3
    logits = torch.randn(B, V, device="cuda") * 3
    wv, wi, nxt = _sample_bufs(B, V)
    seeds = torch.tensor([1, 2, 3], dtype=torch.int64, device="cuda")
    pos = torch.tensor([10, 20, 30], dtype=torch.int32, device="cuda")
    tk = torch.zeros(B, dtype=torch.int32, device="cuda")
    tp = torch.ones(B, device="cuda")
    it = torch.zeros(B, device="cuda")
    ops.sample(logits, it, tk, tp, seeds, pos, nxt, wv, wi)
    assert torch.equal(nxt.cpu(), logits.argmax(-1).to(torch.int32).cpu())
    it = torch.ones(B, device="cuda") / 0.8
    ops.sample(logits, it, tk, tp, seeds, pos, nxt, wv, wi)
    ref = oracle.sample(logits.cpu(), it.cpu(), tk.cpu(), tp.cpu(), seeds.cpu(), pos.cpu())
    for b in range(B):  # same Philox stream; allow fast-math ulps on near ties
        g = oracle.gumbel(int(seeds[b]), torch.tensor([int(nxt[b]), int(ref[b])]), int(pos[b]))
        s_dev = logits[b, nxt[b]].item() * it[b].item() + g[0].item()
        s_ref = logits[b, ref[b]].item() * it[b].item() + g[1].item()
        assert abs(s_dev - s_ref) < 1e-3


def test_sample_topk_topp_and_advance(cuda):
    torch.manual_seed(6)
    B, V = 2, 32000
    logits = torch.randn(B, V, device="cuda") * 2
    wv, wi, nxt = _sample_bufs(B, V)
    seeds = torch.tensor([7, 8], dtype=torch.int64, device="cuda")
    it = torch.ones(B, device="cuda")
    tk = torch.tensor([1, 50], dtype=torch.int32, device="cuda")
    tp = torch.tensor([1.0, 0.9], device="cuda")
    pos = torch.tensor([5, 6], dtype=torch.int32, device="cuda")
    bt = torch.arange(8, dtype=torch.int32, device="cuda").view(2, 4)
    tin = torch.zeros(B, dtype=torch.int32, device="cuda")
    sl = torch.zeros(B, dtype=torch.int32, device="cuda")
    slots = torch.zeros(B, dtype=torch.int32, device="cuda")
    ot = torch.zeros(B, 8, dtype=torch.int32, device="cuda")
    oc = torch.zeros(B, dtype=torch.int32, device="cuda")
    ops.sample(logits, it, tk, tp, seeds, pos, nxt, wv, wi, tokens_in=tin, seq_lens=sl, slots=slots,
               block_tables=bt, bs=4, out_tokens=ot, out_count=oc, use_topkp=True)
    n = nxt.cpu()
    assert int(n[0]) == int(logits[0].argmax())
    top50 = set(torch.topk(logits[1], 50).indices.cpu().tolist())
    assert int(n[1]) in top50
    assert pos.cpu().tolist() == [6, 7] and sl.cpu().tolist() == [7, 8]
    assert slots.cpu().tolist() == [int(bt[0, 1]) * 4 + 2, int(bt[1, 1]) * 4 + 3]
    assert oc.cpu().tolist() == [1, 1] and ot[:, 0].cpu().tolist() == n.tolist() and tin.cpu().tolist() == n.tolist()


@pytest.mark.parametrize("T", [1, 3, 300, 1100])
def test_moe(cuda, T):
    torch.manual_seed(7)
    E, k, H, I = 8, 2, 256, 384
    x = rnd(T, H)
    wgu = rnd(E, 2 * I, H, scale=0.05)
    wd = rnd(E, H, I, scale=0.05)
    logits = torch.randn(T, E, device="cuda")
    w = torch.empty(T, k, device="cuda")
    ids = torch.empty(T, k, dtype=torch.int32, device="cuda")
    ops.moe_route(logits, k, w, ids)
    rw, rids = oracle.moe_route(logits.cpu(), k)
    assert torch.equal(ids.cpu(), rids)
    close(w, rw, 1e-4, 1e-4)
    h = rnd(T, H)
    href = h.cpu().clone()
    oracle.moe_ffn(x.cpu(), wgu.cpu(), wd.cpu(), w.cpu(), ids.cpu(), href)
    if T <= 4:
        act = torch.empty(T * k, I, dtype=BF, device="cuda")
        ops.moe_gemv(x, wgu, ids, k, act, 2 * I, H, ops.EPI_SILU)
        y = torch.empty(T * k, H, dtype=BF, device="cuda")
        ops.moe_gemv(act, wd, ids, 1, y, H, I, ops.EPI_BF16)
    else:
        tile = ops.moe_tile(T * k, E)
        assert tile == (256 if T * k >= 256 * E else 128)
        mt = ops.moe_max_tiles(T * k, E, tile)
        sr = torch.empty(mt * tile, dtype=torch.int32, device="cuda")
        te = torch.empty(mt, dtype=torch.int32, device="cuda")
        tc = torch.empty(1, dtype=torch.int32, device="cuda")
        ops.moe_align(ids, E, sr, te, tc, tile=tile)
        act = torch.empty(T * k, I, dtype=BF, device="cuda")
        ops.moe_gemm(x, wgu, sr, te, tc, act, 2 * I, H, mt, k, epi=ops.EPI_SILU, tile=tile)
        y = torch.empty(T * k, H, dtype=BF, device="cuda")
        ops.moe_gemm(act, wd, sr, te, tc, y, H, I, mt, 1, tile=tile)
    ops.moe_combine(y, w, ids, h)
    close(h, href, 3e-2)


@pytest.mark.parametrize("n,Ts", [(2, 5), (2, 300), (4, 700), (8, 64)])
def test_moe_expert_parallel_prefill_dispatch(cuda, n, Ts):
    """The expert-parallel prefill dispatch on the device (engine ``_moe_ep_a2a``, C4) with n ranks
    emulated on one GPU: per rank the router ids -> ``moe_ep_dispatch`` (stable slots per owner rank,
    -1 padding, no host sync) -> ``gather_rows`` send buffer -> (the all-to-all as a block
    transpose) -> every owner's grouped expert GEMMs over the received rows (``moe_align`` skips the
    -1 padding) -> back -> ``moe_combine`` through the pair slots, against the fp32 oracle of the
    whole MoE layer per token shard. The plan itself must equal the oracle plan exactly."""
    torch.manual_seed(21 + n)
    E, k, H, I = 8, 2, 256, 384
    El = E // n
    wgu = rnd(E, 2 * I, H, scale=0.05)
    wd = rnd(E, H, I, scale=0.05)
    cap = Ts * k
    xs, ws, idss, plans, hs, hrefs = [], [], [], [], [], []
    for r in range(n):
        x = rnd(Ts, H)
        bias = torch.zeros(E, device="cuda")
        bias[r * El] = 3.0 if r == 0 else 0.0  # rank 0's tokens mostly pick its own first expert
        logits = torch.randn(Ts, E, device="cuda") + bias
        w = torch.empty(Ts, k, device="cuda")
        ids = torch.empty(Ts, k, dtype=torch.int32, device="cuda")
        ops.moe_route(logits, k, w, ids)
        plan = ops.moe_ep_dispatch(ids, El, n, cap)
        ref_plan = oracle.moe_ep_dispatch(ids.cpu(), El, n, cap)
        for got, want in zip(plan, ref_plan):
            assert torch.equal(got.cpu(), want), (r, got, want)
        h = rnd(Ts, H)
        href = h.cpu().clone()
        oracle.moe_ffn(x.cpu(), wgu.cpu(), wd.cpu(), w.cpu(), ids.cpu(), href)
        xs.append(x), ws.append(w), idss.append(ids), plans.append(plan), hs.append(h), hrefs.append(href)
    send_x = [ops.gather_rows(xs[r], plans[r][0], k) for r in range(n)]
    for r in range(n):  # padding rows are zeros, real rows the token's x
        sp = plans[r][0].long()
        real = sp >= 0
        assert torch.equal(send_x[r][real], xs[r][sp[real] // k]) and not send_x[r][~real].any()
    y_recv = []
    for d in range(n):  # owner d: rows [d*cap, (d+1)*cap) of every rank's send buffer
        rx = torch.cat([send_x[r][d * cap:(d + 1) * cap] for r in range(n)])
        re = torch.cat([plans[r][1][d * cap:(d + 1) * cap] for r in range(n)]).view(-1, 1)
        P = rx.shape[0]
        tile = ops.moe_tile(P, El)
        mt = ops.moe_max_tiles(P, El, tile)
        sr = torch.empty(mt * tile, dtype=torch.int32, device="cuda")
        te = torch.empty(mt, dtype=torch.int32, device="cuda")
        tc = torch.empty(1, dtype=torch.int32, device="cuda")
        ops.moe_align(re, El, sr, te, tc, tile=tile)
        act = torch.empty(P, I, dtype=BF, device="cuda")
        ops.moe_gemm(rx, wgu[d * El:(d + 1) * El].contiguous(), sr, te, tc, act, 2 * I, H, mt, 1, epi=ops.EPI_SILU,
                     tile=tile)
        y = torch.full((P, H), float("nan"), dtype=BF, device="cuda")
        ops.moe_gemm(act, wd[d * El:(d + 1) * El].contiguous(), sr, te, tc, y, H, I, mt, 1, tile=tile)
        y_recv.append(y)
    for r in range(n):
        y_back = torch.cat([y_recv[d][r * cap:(r + 1) * cap] for d in range(n)])
        ops.moe_combine(y_back, ws[r], idss[r], hs[r], rows=plans[r][2])
        close(hs[r], hrefs[r], 3e-2)


@pytest.mark.parametrize("T,tile", [(700, 128), (1500, 256), (2600, 256)])
def test_moe_grouped_gemm_ragged(cuda, T, tile):
    """The grouped expert GEMM on ragged groups: the router is skewed so two experts take most
    pairs (hundreds of rows each, several 256-row tiles, a partial last tile) and others a few;
    gate_up (SiLU-mul in the epilogue) and down per pair vs an fp32 per-expert oracle."""
    torch.manual_seed(11)
    E, k, H, I = 8, 2, 512, 640
    x = rnd(T, H)
    wgu = rnd(E, 2 * I, H, scale=0.05)
    wd = rnd(E, H, I, scale=0.05)
    logits = torch.randn(T, E, device="cuda") + torch.tensor([3.0, 2.5, 0, 0, -1, -2, -3, -4], device="cuda")
    w = torch.empty(T, k, device="cuda")
    ids = torch.empty(T, k, dtype=torch.int32, device="cuda")
    ops.moe_route(logits, k, w, ids)
    counts = torch.bincount(ids.view(-1).long().cpu(), minlength=E)
    assert counts.max() > 2 * 128 and counts.min() < 128, counts  # ragged: big groups and small ones
    assert ops.moe_tile(T * k, E) == tile
    mt = ops.moe_max_tiles(T * k, E, tile)
    sr = torch.empty(mt * tile, dtype=torch.int32, device="cuda")
    te = torch.empty(mt, dtype=torch.int32, device="cuda")
    tc = torch.empty(1, dtype=torch.int32, device="cuda")
    ops.moe_align(ids, E, sr, te, tc, tile=tile)
    act = torch.full((T * k, I), float("nan"), dtype=BF, device="cuda")
    ops.moe_gemm(x, wgu, sr, te, tc, act, 2 * I, H, mt, k, epi=ops.EPI_SILU, tile=tile)
    y = torch.full((T * k, H), float("nan"), dtype=BF, device="cuda")
    ops.moe_gemm(act, wd, sr, te, tc, y, H, I, mt, 1, tile=tile)
    # fp32 oracle per expert group (every pair written: NaN poison would show a missed row)
    xr, idc = x.float().repeat_interleave(k, 0), ids.view(-1).long()
    aref = torch.empty(T * k, I, device="cuda")
    yref = torch.empty(T * k, H, device="cuda")
    for e in range(E):
        sel = (idc == e).nonzero().view(-1)
        g = xr[sel] @ wgu[e].float().t()
        aref[sel] = torch.nn.functional.silu(g[:, 0::2]) * g[:, 1::2]
        yref[sel] = act[sel].float() @ wd[e].float().t()
    close(act, aref, 3e-2)
    close(y, yref, 3e-2)


@pytest.mark.parametrize("T,E,H", [(1, 8, 4096), (4, 8, 256), (2, 16, 1024), (3, 4, 192)])
def test_moe_router_fused(cuda, T, E, H):
    """Decode router in one launch (rmsnorm -> router GEMV -> softmax top-k) vs the fp32 oracle, and
    the expert gate_up GEMV normalising raw hidden rows in its prologue vs normed rows."""
    torch.manual_seed(9)
    k = 2
    h = rnd(T, H)
    nw = (1 + 0.1 * torch.randn(H, device="cuda")).to(BF)
    wr = rnd(E, H, scale=0.05)
    w = torch.empty(T, k, device="cuda")
    ids = torch.empty(T, k, dtype=torch.int32, device="cuda")
    ops.moe_router(h, nw, 1e-5, wr, k, w, ids)
    xn = oracle.rmsnorm(h.cpu(), nw.cpu(), 1e-5)
    logits = oracle.linear(xn, wr.cpu(), ops.EPI_F32)
    rw, rids = oracle.moe_route(logits, k)
    # a near-tie of the logits may order two experts differently: compare the selected sets' logits
    got = torch.gather(logits, 1, ids.cpu().long())
    ref = torch.gather(logits, 1, rids.long())
    close(got, ref, 1e-3, 1e-3)
    close(w, rw, 2e-3, 2e-3)
    I = 384
    wgu = rnd(E, 2 * I, H, scale=0.05)
    a1 = torch.empty(T * k, I, dtype=BF, device="cuda")
    a2 = torch.empty(T * k, I, dtype=BF, device="cuda")
    ops.moe_gemv(h, wgu, ids, k, a1, 2 * I, H, ops.EPI_SILU, norm_w=nw, eps=1e-5)
    ops.moe_gemv(xn.to(h.device), wgu, ids, k, a2, 2 * I, H, ops.EPI_SILU)
    close(a1, a2, 2e-2)
    # down projection + combine in one launch vs an fp32 reference (the unfused path rounds each
    # expert output to bf16 before the combine, so it is the less exact one)
    wd = rnd(E, H, I, scale=0.05)
    h1 = h.clone()
    ops.moe_down_combine(a1, wd, ids, w, h1, H, I)
    href = h.float().cpu().clone()
    a1c, wdc, idc, wc = a1.float().cpu(), wd.float().cpu(), ids.cpu().long(), w.cpu()
    for t in range(T):
        for j in range(k):
            href[t] += wc[t, j] * (wdc[idc[t, j]] @ a1c[t * k + j])
    close(h1, href, 2e-2)


@pytest.mark.parametrize("T,E,H,k", [(1, 8, 4096, 2), (37, 8, 4096, 2), (2048, 8, 4096, 2), (300, 16, 1024, 4),
                                     (129, 4, 192, 2)])
def test_moe_route_fused(cuda, T, E, H, k):
    """The one-launch prefill router (logits in f32 from the bf16 rows, softmax, top-k, renormalise)
    vs the fp32 oracle: the same experts wherever the oracle's k-th and (k+1)-th logits are not a
    near-tie, weights to f32 rounding."""
    torch.manual_seed(31)
    x = rnd(T, H)
    wr = rnd(E, H, scale=0.05)
    w = torch.empty(T, k, device="cuda")
    ids = torch.empty(T, k, dtype=torch.int32, device="cuda")
    ops.moe_route_fused(x, wr, k, w, ids)
    logits = x.float().cpu() @ wr.float().cpu().t()
    rw, rids = oracle.moe_route(logits, k)
    srt = logits.sort(dim=-1, descending=True).values
    clear = (srt[:, k - 1] - srt[:, k]) > 1e-3 * srt.abs().max()
    if k > 1:
        clear &= ((srt[:, :k - 1] - srt[:, 1:k]).abs() > 1e-3 * srt.abs().max()).all(-1)
    assert clear.float().mean() > 0.9
    assert torch.equal(ids.cpu()[clear], rids[clear])
    close(w[clear.cuda()], rw[clear], 1e-4, 1e-3)
