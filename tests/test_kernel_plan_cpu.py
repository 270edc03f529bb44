"""Host-side launch planning of the HIP kernels (no GPU: the planners are plain C++ in the kernel
library). Prefill attention KV split, csrc/kernels/attn_prefill.hip ``llmc_attn_prefill_plan``."""

import pytest

from llm_consensus_amd import ops


@pytest.mark.parametrize("B,T,ctx,nh,nkv,split", [
    (1, 8192, 8192, 4, 1, 4),         # a TP=8 rank: one kv head, 128 blocks -> 4 ways (1.7x measured)
    (1, 2048, 2048, 4, 1, 4),
    (1, 8192, 8192, 8, 1, 2),         # 256 blocks of up to 128 tiles: 2 ways (1.3x)
    (1, 2048, 2048, 16, 2, 2),        # 64 blocks: 2 ways (1.15x)
    (1, 2048, 2048, 32, 8, 1),        # 256 blocks of 1..32 tiles: a split costs more than it saves
    (1, 8192, 8192, 32, 8, 1),        # 1024 blocks: the longest-first order balances already
    (4, 8192, 8192, 32, 8, 1),
    (1, 256, 256, 32, 8, 1),          # 4 key tiles: nothing worth sharing
])
def test_prefill_split_plan(B, T, ctx, nh, nkv, split):
    k, kmin = ops.attn_prefill_plan(B, T, ctx, nh, nkv, ksplit=-1)
    assert k == split, (k, kmin)
    if k > 1:
        assert 1 <= kmin <= (ctx + 63) // 64 // 2  # some group is long enough to split


def test_prefill_split_overrides():
    assert ops.attn_prefill_plan(1, 2048, 2048, 32, 8, ksplit=1)[0] == 1
    assert ops.attn_prefill_plan(1, 2048, 2048, 32, 8, ksplit=4, kmin=3) == (4, 3)
    assert ops.attn_prefill_plan(1, 2048, 2048, 32, 8, ksplit=99, kmin=3) == (4, 3)
