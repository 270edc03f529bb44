"""Decoder-only transformer weights for the Llama-3 / Mixtral / Phi-3 families (T1).

All three families share one engine-facing layout, chosen for the kernels rather than for
checkpoint compatibility:
  * ``w_qkv``  [q + 2 kv, H]  fused Q|K|V rows (one GEMV/GEMM per layer); inside every Q and
    K head the rows are PAIR-INTERLEAVED (row 2i = dim i, row 2i + 1 = dim i + D/2) so the
    rotate-half RoPE pair of a head lands in one wave of the decode GEMV, whose epilogue applies
    RoPE and writes K/V straight into the paged cache (no separate RoPE launch);
  * ``w_o``    [H, q];
  * ``w_gu``   [2 I, H] gate/up rows INTERLEAVED (row 2i = gate_i, 2i + 1 = up_i) so the GEMV
    epilogue produces silu(gate) * up directly and a TP shard is a contiguous row range;
  * ``w_down`` [H, I];
  * MoE (Mixtral): ``w_router`` [E, H], ``w_gu`` [E, 2I, H], ``w_down`` [E, H, I] (under TP: 1/tp
    of every expert's FFN rows, or with ``expert_parallel`` E/tp whole experts per rank);
  * ``embed`` [V, H] (replicated under TP), ``lm_head`` [V, H] (vocab-parallel under TP).
Weights are random-init from a seed, or read from a Hugging Face checkpoint when the config
names one (``models/checkpoint.py``). Either way each tensor is produced in full in the logical
layout (from its own (seed, name)-derived generator, or from the safetensors shards) and then
sliced to this rank's shard, so TP=1 and TP=n models are the SAME model (tested on CPU with gloo).
"""

from __future__ import annotations

import math
import zlib
from typing import List, Optional

import torch

from ..parallel.comm import TPGroup, shard_range
from .config import ModelConfig


class LayerWeights:
    __slots__ = ("ln1", "ln2", "w_qkv", "w_o", "w_gu", "w_down", "w_router")

    def __init__(self):
        for s in self.__slots__:
            setattr(self, s, None)


class TransformerWeights:
    def __init__(self, cfg: ModelConfig, tp: TPGroup, device: torch.device, seed: int,
                 init_scale: float = 1.0, source=None, expert_parallel: bool = False):
        if source is None and cfg.checkpoint:
            from .checkpoint import HFCheckpoint

            source = HFCheckpoint(cfg.checkpoint, cfg)
        self.source = source
        self.cfg = cfg
        self.tp = tp
        self.device = device
        self.seed = seed
        self.init_scale = init_scale
        if cfg.n_heads % tp.size or cfg.n_kv_heads % tp.size or cfg.intermediate % tp.size or cfg.vocab % tp.size:
            raise ValueError(f"{cfg.name}: not shardable with tp={tp.size}")
        # expert parallel (MoE under TP): whole experts [e0, e0 + n_local_experts) on this rank
        self.ep = bool(expert_parallel and cfg.is_moe and tp.size > 1)
        if self.ep and cfg.n_experts % tp.size:
            raise ValueError(f"{cfg.name}: {cfg.n_experts} experts not shardable over ep={tp.size}")
        self.n_local_experts = cfg.n_experts // tp.size if self.ep else cfg.n_experts
        self.e0 = tp.rank * self.n_local_experts if self.ep else 0
        self.nh = cfg.n_heads // tp.size
        self.nkv = cfg.n_kv_heads // tp.size
        self.inter = cfg.intermediate if self.ep else cfg.intermediate // tp.size
        self.vocab_local = cfg.vocab // tp.size
        self.q_size = self.nh * cfg.head_dim
        self.kv_size = self.nkv * cfg.head_dim
        self.qkv_size = self.q_size + 2 * self.kv_size
        self.layers: List[LayerWeights] = []
        self._build()
        self.source = None  # release the checkpoint's file handles

    # -- generation -------------------------------------------------------------------------
    def _gen(self, name: str, shape, std: float, mean: float = 0.0) -> torch.Tensor:
        s = (zlib.crc32(name.encode()) ^ (self.seed * 0x9E3779B1)) & 0x7FFFFFFFFFFF
        g = torch.Generator(device=self.device)
        g.manual_seed(s)
        t = torch.randn(*shape, generator=g, device=self.device, dtype=torch.float32)
        if std != 1.0:
            t.mul_(std)
        if mean != 0.0:
            t.add_(mean)
        return t.to(torch.bfloat16)

    def _full(self, name: str, shape, kind: str = "linear") -> torch.Tensor:
        """Full (unsharded) logical tensor ``name``: checkpoint or seeded random init."""
        if self.source is not None:
            t = self.source.get(name)
            if tuple(t.shape) != tuple(shape):
                raise ValueError(f"checkpoint tensor {name}: shape {tuple(t.shape)} != expected {tuple(shape)}")
            return t.to(device=self.device, dtype=torch.bfloat16)
        if kind == "embed":
            return self._gen(name, shape, 1.0)
        if kind == "norm":
            return self._gen(name, shape, 0.02, 1.0)
        return self._gen(name, shape, self.init_scale / math.sqrt(shape[1]))

    def _linear(self, name: str, n_out: int, n_in: int) -> torch.Tensor:
        return self._full(name, (n_out, n_in))

    def _build(self) -> None:
        c, r, n = self.cfg, self.tp.rank, self.tp.size
        D = c.head_dim
        with torch.no_grad():
            self.embed = self._full("embed", (c.vocab, c.hidden), "embed")
            self.final_norm = self._full("final_norm", (c.hidden,), "norm")
            lm = self._linear("lm_head", c.vocab, c.hidden)
            v0, v1 = shard_range(c.vocab, r, n)
            self.lm_head = lm[v0:v1].contiguous()
            del lm
            for i in range(c.n_layers):
                L = LayerWeights()
                p = f"layers.{i}."
                L.ln1 = self._full(p + "ln1", (c.hidden,), "norm")
                L.ln2 = self._full(p + "ln2", (c.hidden,), "norm")
                qkv = self._linear(p + "w_qkv", c.qkv_size, c.hidden)
                q0, q1 = shard_range(c.n_heads, r, n)
                k0, k1 = shard_range(c.n_kv_heads, r, n)
                qs = qkv[q0 * D:q1 * D]
                ks = qkv[c.q_size + k0 * D:c.q_size + k1 * D]
                vs = qkv[c.q_size + c.kv_size + k0 * D:c.q_size + c.kv_size + k1 * D]
                L.w_qkv = torch.cat([pair_interleave_heads(qs, D), pair_interleave_heads(ks, D), vs], 0).contiguous()
                del qkv
                wo = self._linear(p + "w_o", c.hidden, c.q_size)
                L.w_o = wo[:, q0 * D:q1 * D].contiguous()
                del wo
                i0, i1 = shard_range(c.intermediate, r, n)
                if c.is_moe:
                    L.w_router = self._linear(p + "w_router", c.n_experts, c.hidden)
                    gus, downs = [], []
                    for e in range(self.e0, self.e0 + self.n_local_experts):
                        gu = self._linear(p + f"experts.{e}.w_gu", 2 * c.intermediate, c.hidden)
                        dn = self._linear(p + f"experts.{e}.w_down", c.hidden, c.intermediate)
                        if self.ep:  # whole experts
                            gus.append(gu)
                            downs.append(dn)
                        else:        # every expert, 1/tp of its FFN rows
                            gus.append(gu[2 * i0:2 * i1])
                            downs.append(dn[:, i0:i1])
                    L.w_gu = torch.stack(gus).contiguous()
                    L.w_down = torch.stack(downs).contiguous()
                    del gus, downs
                else:
                    gu = self._linear(p + "w_gu", 2 * c.intermediate, c.hidden)
                    L.w_gu = gu[2 * i0:2 * i1].contiguous()
                    del gu
                    dn = self._linear(p + "w_down", c.hidden, c.intermediate)
                    L.w_down = dn[:, i0:i1].contiguous()
                    del dn
                self.layers.append(L)

    def to(self, device) -> "TransformerWeights":
        """Move every tensor (in place) to ``device``; returns self."""
        device = torch.device(device)
        self.device = device
        self.embed = self.embed.to(device)
        self.final_norm = self.final_norm.to(device)
        self.lm_head = self.lm_head.to(device)
        for L in self.layers:
            for s in LayerWeights.__slots__:
                t = getattr(L, s)
                if t is not None:
                    setattr(L, s, t.to(device))
        return self

    def nbytes(self) -> int:
        tot = self.embed.numel() + self.final_norm.numel() + self.lm_head.numel()
        for L in self.layers:
            for s in LayerWeights.__slots__:
                t = getattr(L, s)
                if t is not None:
                    tot += t.numel()
        return tot * 2


def pair_interleave_heads(rows: torch.Tensor, D: int) -> torch.Tensor:
    """Reorder each head's D rows as [0, D/2, 1, D/2 + 1, ...] (see module docstring)."""
    n = rows.shape[0] // D
    half = D // 2
    r = rows.view(n, 2, half, -1).transpose(1, 2)  # [head, i, {i, i+half}, H]
    return r.reshape(n * D, -1)


def full_reference_weights(cfg: ModelConfig, seed: int, device="cpu", init_scale: float = 1.0) -> TransformerWeights:
    return TransformerWeights(cfg, TPGroup.single(), torch.device(device), seed, init_scale)


def split_for_rank(full: Optional[TransformerWeights], cfg: ModelConfig, tp: TPGroup, device, seed: int,
                   init_scale: float = 1.0) -> TransformerWeights:
    return TransformerWeights(cfg, tp, torch.device(device), seed, init_scale)
