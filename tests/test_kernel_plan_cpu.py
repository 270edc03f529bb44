"""Host-side launch planning of the HIP kernels (no GPU: the planners are plain C++ in the kernel
library). Prefill attention KV split, csrc/kernels/attn_prefill.hip ``llmc_attn_prefill_plan``; prefill
GEMM kernel choice, csrc/kernels/gemm.hip ``llmc_gemm_plan``."""

import pytest

from llm_consensus_amd import ops


@pytest.mark.parametrize("B,T,ctx,nh,nkv,split", [
    (1, 8192, 8192, 4, 1, 4),         # a TP=8 rank: one kv head, 128 blocks -> 4 ways (134-142 us vs key halves 157)
    (1, 2048, 2048, 4, 1, 1),         # the unsplit key-halves form: 41.2 us vs 4 ways 50.7
    (1, 4096, 4096, 4, 1, 1),         # 73.7 vs 2 ways 81.4
    (1, 8192, 8192, 8, 1, 1),         # 175 vs 2 ways 191.6
    (1, 4096, 4096, 8, 2, 1),         # 75.5 vs 2 ways 85.9
    (1, 2048, 2048, 16, 2, 1),        # 42.8 vs 2 ways 61.5
    (1, 2048, 2048, 32, 8, 1),        # 256 blocks of 1..32 tiles: the paired form
    (1, 8192, 8192, 32, 8, 1),        # 1024 blocks: the longest-first order balances already
    (4, 8192, 8192, 32, 8, 1),
    (1, 256, 256, 32, 8, 1),          # 4 key tiles: nothing worth sharing
])
def test_prefill_split_plan(B, T, ctx, nh, nkv, split):
    k, kmin = ops.attn_prefill_plan(B, T, ctx, nh, nkv, ksplit=-1)
    if split == 4:  # without the key-halves form (D = 96 / other page sizes) the 0.80 bar applies
        assert ops.attn_prefill_plan(B, T, ctx, nh, nkv, ksplit=-1, D=96)[0] == 4
    assert k == split, (k, kmin)
    if k > 1:
        assert 1 <= kmin <= (ctx + 63) // 64 // 2  # some group is long enough to split


@pytest.mark.parametrize("B,T,nh,nkv", [(1, 8192, 4, 1), (2, 300, 32, 8), (1, 33, 32, 32), (3, 2048, 16, 2)])
def test_prefill_split_counters_match_the_kernel_grid(B, T, nh, nkv):
    """one counter per (sequence, row-tile group of the 8-wave split grid, kv head) —
    ngrp = ceil(G * ceil(T / 32) / 8), the kernel's gridDim.x / nkv / ksplit — from one helper that
    both the workspace and the launch check use."""
    G, npb = nh // nkv, (T + 31) // 32
    assert ops.attn_prefill_counters(B, T, nh, nkv) == B * ((G * npb + 7) // 8) * nkv
    assert ops.attn_prefill_workspace(2, T, nh, 128, "cpu", B, nkv, T)[1].numel() == B * ((G * npb + 7) // 8) * nkv


def test_prefill_split_overrides():
    assert ops.attn_prefill_plan(1, 2048, 2048, 32, 8, ksplit=1)[0] == 1
    assert ops.attn_prefill_plan(1, 2048, 2048, 32, 8, ksplit=4, kmin=3) == (4, 3)
    assert ops.attn_prefill_plan(1, 2048, 2048, 32, 8, ksplit=99, kmin=3) == (4, 3)


@pytest.mark.parametrize("B,T,nh,nkv,ksplit,form", [
    (1, 2048, 32, 8, 1, 1),     # Llama-3-8B 2k: 256 8-wave blocks = one round, G <= 4 -> paired (76.6 -> 58.5 us)
    (1, 2048, 32, 32, 1, 1),    # 69.9 -> 57.0
    (1, 1024, 32, 8, 1, 3),     # 128 blocks: key halves (39.5 -> 27.8)
    (1, 2048, 16, 2, 1, 3),     # G = 8 (70B TP=4 rank): no pairs; key halves (72.1 -> 42.8)
    (1, 4096, 16, 2, 1, 3),     # 256 blocks, G = 8: key halves (129.3 -> 92.1)
    (1, 8192, 32, 8, 1, 0),     # 1024 blocks: the 8-wave longest-first grid
    (2, 2048, 32, 8, 1, 0),     # two sequences: 512 blocks
    (1, 8192, 16, 2, 1, 0),     # 512 blocks
    (1, 8192, 4, 1, 4, 0),      # a split grid
])
def test_prefill_block_form(B, T, nh, nkv, ksplit, form):
    from llm_consensus_amd.ops import kernels
    assert kernels().attn_prefill_form(B, T, nh, nkv, ksplit, 128, 64) == form
    if form == 3:  # key halves need D = 128 on 64-key pages: otherwise 4-wave blocks
        assert kernels().attn_prefill_form(B, T, nh, nkv, ksplit, 96, 64) == 2


@pytest.mark.parametrize("M,N,kind", [
    (8192, 768, "128x192"),    # a TP=8 rank's qkv: 96 tiles of 256 x 256 for 256 CUs (53.5 vs 81.5 us)
    (2048, 768, "128x192"),
    (3425, 768, "128x192"),    # the N=8 bench's judge prompt on a TP=8 rank
    (33000, 768, "256x256"),   # 2 rounds of 256 x 256 against 5 of 128 x 192 (188 vs 259 us)
    (8192, 6144, "256x256"),   # Llama-3-8B qkv / o / gate_up: full rounds of 256 x 256
    (8192, 4096, "256x256"),
    (8192, 2560, "256x256"),   # 70B TP=4 qkv: 2 rounds against 4 (330 vs 366 us)
    (8192, 28672, "256x256"),
])
def test_gemm_plan(M, N, kind):
    assert ops.gemm_plan(M, N) == kind


def test_every_kernel_launch_has_its_host_stub():
    """Each <<<>>> launch needs the kernel's host-side stub in the library. hipcc drops a template
    kernel's stub WITHOUT a diagnostic when a target builtin in it takes a template-dependent operand
    type (round 5: the narrow GEMM's per-lane offset array sized by the template parameter); the
    library then links and fails at import on the GPU box with an undefined symbol."""
    import glob
    import os
    import shutil
    import subprocess

    nm = shutil.which("nm")
    if nm is None:
        pytest.skip("nm not on PATH")
    lib = os.path.join(os.path.dirname(ops.__file__), "..", "_lib")
    libs = glob.glob(os.path.join(lib, "_llmc_hip*.so"))
    assert libs, "kernel library not built"
    out = subprocess.run([nm, "-D", libs[0]], capture_output=True, text=True, check=True).stdout
    missing = [ln.split()[-1] for ln in out.splitlines() if ln.split()[:1] == ["U"] and "__device_stub__" in ln]
    assert not missing, missing


def _kernel_scratch_bytes():
    """{kernel symbol: private segment bytes per lane} of every gfx950 kernel in the built library:
    the .hip_fatbin section holds one offload bundle per source file; each device code object's
    metadata note pairs .private_segment_fixed_size with .symbol (keys sorted within a kernel)."""
    import glob
    import os
    import subprocess
    import tempfile

    tools = "/opt/rocm/lib/llvm/bin"
    if not all(os.path.exists(os.path.join(tools, t)) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")):
        pytest.skip("ROCm LLVM tools not found")
    libs = glob.glob(os.path.join(os.path.dirname(ops.__file__), "..", "_lib", "_llmc_hip*.so"))
    assert libs, "kernel library not built"
    res = {}
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin")
        subprocess.run([f"{tools}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", libs[0]], check=True)
        data = open(fb, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        offs, i = [], data.find(magic)
        while i >= 0:
            offs.append(i)
            i = data.find(magic, i + 1)
        for k, o in enumerate(offs):
            bundle, co = os.path.join(d, f"b{k}"), os.path.join(d, f"c{k}.elf")
            with open(bundle, "wb") as f:
                f.write(data[o:offs[k + 1] if k + 1 < len(offs) else len(data)])
            r = subprocess.run([f"{tools}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={bundle}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
            if r.returncode != 0:
                continue
            notes = subprocess.run([f"{tools}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
            pending = None
            for ln in notes.splitlines():
                ln = ln.strip()
                if ln.startswith(".private_segment_fixed_size:"):
                    pending = int(ln.split(":")[1])
                elif ln.startswith(".symbol:") and pending is not None:
                    res[ln.split(":", 1)[1].strip()] = pending
                    pending = None
    return res


def test_no_kernel_uses_scratch():
    """No gfx950 kernel of the library keeps per-lane state in scratch (a silent 10x slowdown: a
    refactor of the prefill tile loop into lambdas called from three loops put their captures on the
    stack, 640 B per lane, with vgpr_spill_count still 0; the 3-4-row, 8-loads-per-lane VALU GEMV
    with the RMS-norm prologue kept 20-48 B and is no longer instantiated)."""
    res = _kernel_scratch_bytes()
    assert len(res) > 100, len(res)
    bad = {k: v for k, v in res.items() if v}
    assert not bad, bad
