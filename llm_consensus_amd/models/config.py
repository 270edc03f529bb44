"""Architecture configs of the on-node model families (SURVEY.md §2.6 model shapes).

Weights are random-init (seeded per replica): there is no network to fetch checkpoints, and the
benchmark contract is "random-init weights of that architecture". Shapes are the public configs.
"""

from __future__ import annotations

import dataclasses
import math
from typing import Optional


@dataclasses.dataclass(frozen=True)
class RopeScaling:
    """Llama-3.1-style frequency-dependent RoPE scaling (for a judge context beyond 8k)."""

    factor: float = 8.0
    low_freq_factor: float = 1.0
    high_freq_factor: float = 4.0
    original_max_position: int = 8192


@dataclasses.dataclass(frozen=True)
class ModelConfig:
    name: str
    arch: str  # "llama" | "mixtral" | "phi3"
    n_layers: int
    hidden: int
    n_heads: int
    n_kv_heads: int
    head_dim: int
    intermediate: int
    vocab: int
    rope_theta: float
    rms_eps: float = 1e-5
    max_position: int = 8192
    n_experts: int = 0
    top_k_experts: int = 0
    rope_scaling: Optional[RopeScaling] = None
    default_tp: int = 1
    # Hugging Face checkpoint directory (models/checkpoint.py); None = seeded random init
    checkpoint: Optional[str] = None
    bos_id: int = -1            # -1: the synthetic tokenizer's (vocab - 2)
    eos_ids: tuple = ()         # empty: the synthetic tokenizer's (vocab - 1)
    tie_embeddings: bool = False

    @property
    def eos(self) -> tuple:
        return self.eos_ids or (self.vocab - 1,)

    # -- derived sizes ---------------------------------------------------------------------
    @property
    def q_size(self) -> int:
        return self.n_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.n_kv_heads * self.head_dim

    @property
    def qkv_size(self) -> int:
        return self.q_size + 2 * self.kv_size

    @property
    def is_moe(self) -> bool:
        return self.n_experts > 0

    def num_params(self) -> int:
        h, i = self.hidden, self.intermediate
        attn = h * self.qkv_size + self.q_size * h
        mlp = 3 * h * i * (self.n_experts if self.is_moe else 1)
        router = h * self.n_experts if self.is_moe else 0
        per_layer = attn + mlp + router + 2 * h
        return self.n_layers * per_layer + 2 * self.vocab * h + h

    def weight_bytes(self, dtype_bytes: int = 2) -> int:
        return self.num_params() * dtype_bytes

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.n_layers * self.kv_size * dtype_bytes

    def active_weight_bytes(self, dtype_bytes: int = 2) -> int:
        """Bytes streamed per decode token at batch 1 (MoE: top-k experts only)."""
        if not self.is_moe:
            return self.weight_bytes(dtype_bytes) - self.vocab * self.hidden * dtype_bytes  # embed not streamed
        h, i = self.hidden, self.intermediate
        per_layer = h * self.qkv_size + self.q_size * h + 3 * h * i * self.top_k_experts + h * self.n_experts
        return (self.n_layers * per_layer + self.vocab * h) * dtype_bytes

    def with_(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)


LLAMA3_8B = ModelConfig("llama-3-8b", "llama", 32, 4096, 32, 8, 128, 14336, 128256, 500000.0,
                        max_position=131072, rope_scaling=RopeScaling())
LLAMA3_70B = ModelConfig("llama-3-70b", "llama", 80, 8192, 64, 8, 128, 28672, 128256, 500000.0,
                         max_position=131072, rope_scaling=RopeScaling(), default_tp=4)
MIXTRAL_8X7B = ModelConfig("mixtral-8x7b", "mixtral", 32, 4096, 32, 8, 128, 14336, 32000, 1000000.0,
                           max_position=32768, n_experts=8, top_k_experts=2)
PHI3_MINI = ModelConfig("phi-3-mini", "phi3", 32, 3072, 32, 32, 96, 8192, 32064, 10000.0,
                        max_position=4096)

# Tiny variants: same code paths and kernel shape classes (GQA, d=128/96, MoE), small enough
# for CPU tests and fast GPU numerics tests.
LLAMA_TINY = ModelConfig("llama-tiny", "llama", 2, 256, 4, 2, 64, 512, 1024, 500000.0, max_position=4096)
LLAMA_SMALL = ModelConfig("llama-small", "llama", 4, 1024, 8, 2, 128, 2816, 32000, 500000.0, max_position=8192)
MIXTRAL_TINY = ModelConfig("mixtral-tiny", "mixtral", 2, 256, 4, 2, 64, 384, 1024, 1000000.0,
                           max_position=4096, n_experts=4, top_k_experts=2)
PHI3_TINY = ModelConfig("phi3-tiny", "phi3", 2, 192, 2, 2, 96, 384, 1024, 10000.0, max_position=4096)
# tiny stand-in for Llama-3-70B in TP=4 rehearsals (heads, kv heads, FFN and vocab shard over 4)
LLAMA_TINY_TP4 = ModelConfig("llama-tiny-tp4", "llama", 2, 512, 8, 4, 64, 1024, 1024, 500000.0, max_position=16384,
                             default_tp=4)

FAMILIES = {c.name: c for c in (LLAMA3_8B, LLAMA3_70B, MIXTRAL_8X7B, PHI3_MINI,
                                LLAMA_TINY, LLAMA_SMALL, MIXTRAL_TINY, PHI3_TINY, LLAMA_TINY_TP4)}


def rope_inv_freq(cfg: ModelConfig):
    """Inverse frequencies (float64 list) incl. Llama-3.1 scaling; shared by kernels and oracle."""
    d = cfg.head_dim
    inv = [1.0 / (cfg.rope_theta ** (2 * i / d)) for i in range(d // 2)]
    rs = cfg.rope_scaling
    if rs is None:
        return inv
    low_wl = rs.original_max_position / rs.low_freq_factor
    high_wl = rs.original_max_position / rs.high_freq_factor
    out = []
    for f in inv:
        wl = 2 * math.pi / f
        if wl < high_wl:
            out.append(f)
        elif wl > low_wl:
            out.append(f / rs.factor)
        else:
            smooth = (rs.original_max_position / wl - rs.low_freq_factor) / (rs.high_freq_factor - rs.low_freq_factor)
            out.append((1 - smooth) * f / rs.factor + smooth * f)
    return out
