"""Hugging Face checkpoint support: ``config.json`` + ``*.safetensors`` → engine weights.

The reference has no local models at all: every "model" is a remote API (``internal/provider/
{openai,anthropic,google}.go``) and local models are only a wish (``docs/proposed-features.md``).
Here a directory in Hugging Face layout becomes a first-class catalog family
(``--weights-dir``), served by the same engine and kernels as the random-init architectures:

* ``config_from_hf(dir)`` maps ``config.json`` (model_type llama / mixtral / phi3) to a
  :class:`ModelConfig` (Llama-3.1 ``rope_scaling`` included) that records the checkpoint path and
  the tokenizer's BOS / EOS ids;
* :class:`HFCheckpoint` reads tensors lazily (``safetensors.safe_open``; nothing is unpickled) and
  returns them in the engine's *logical* layout (``models/transformer.py``): fused Q|K|V rows,
  gate/up rows interleaved; the caller applies the head pair-interleave and the TP slice, so a
  checkpoint shards exactly like the random-init weights. Both the hub layout of Mixtral
  (``block_sparse_moe.experts.{e}.w1/w2/w3``) and the fused one written by transformers 5
  (``mlp.experts.gate_up_proj``) are understood.

Unsupported checkpoint features (attention/MLP biases, sliding windows shorter than the context,
partial rotary, LongRoPE) raise :class:`CheckpointError` instead of running a wrong model.
"""

from __future__ import annotations

import glob
import json
import os
from typing import Dict, List, Optional

import torch

from .config import FAMILIES, ModelConfig, RopeScaling


class CheckpointError(Exception):
    pass


def _read_json(path: str) -> dict:
    with open(path, encoding="utf-8") as f:
        return json.load(f)


def is_checkpoint_dir(path: str) -> bool:
    return os.path.isfile(os.path.join(path, "config.json")) and bool(glob.glob(os.path.join(path, "*.safetensors")))


def _ids(v) -> List[int]:
    if v is None:
        return []
    return [int(x) for x in v] if isinstance(v, (list, tuple)) else [int(v)]


def config_from_hf(path: str, name: Optional[str] = None) -> ModelConfig:
    """ModelConfig of the Hugging Face checkpoint directory ``path``."""
    hc = _read_json(os.path.join(path, "config.json"))
    mt = hc.get("model_type", "")
    arch = {"llama": "llama", "mixtral": "mixtral", "phi3": "phi3"}.get(mt)
    if arch is None:
        raise CheckpointError(f"{path}: model_type {mt!r} not supported (llama, mixtral, phi3)")
    if hc.get("attention_bias") or hc.get("mlp_bias"):
        raise CheckpointError(f"{path}: attention/MLP biases are not supported")
    if float(hc.get("partial_rotary_factor", 1.0)) != 1.0:
        raise CheckpointError(f"{path}: partial rotary embeddings are not supported")
    heads = int(hc["num_attention_heads"])
    hidden = int(hc["hidden_size"])
    head_dim = int(hc.get("head_dim") or hidden // heads)
    max_pos = int(hc.get("max_position_embeddings", 8192))
    sw = hc.get("sliding_window")
    if sw is not None and int(sw) < max_pos:
        raise CheckpointError(f"{path}: sliding-window attention ({sw}) is not supported")
    rp = hc.get("rope_parameters") or {}
    theta = float(hc.get("rope_theta") or rp.get("rope_theta") or 10000.0)
    rs_cfg = hc.get("rope_scaling") or (rp if rp.get("rope_type") not in (None, "default") else None)
    scaling = None
    if rs_cfg:
        kind = rs_cfg.get("rope_type") or rs_cfg.get("type")
        if kind != "llama3":
            raise CheckpointError(f"{path}: rope scaling {kind!r} is not supported (llama3 only)")
        scaling = RopeScaling(float(rs_cfg["factor"]), float(rs_cfg.get("low_freq_factor", 1.0)),
                              float(rs_cfg.get("high_freq_factor", 4.0)),
                              int(rs_cfg.get("original_max_position_embeddings", 8192)))
    bos, eos = _ids(hc.get("bos_token_id")), _ids(hc.get("eos_token_id"))
    gen = os.path.join(path, "generation_config.json")
    if os.path.isfile(gen):
        eos = _ids(_read_json(gen).get("eos_token_id")) or eos
    vocab = int(hc["vocab_size"])
    return ModelConfig(
        name=name or os.path.basename(os.path.normpath(path)),
        arch=arch,
        n_layers=int(hc["num_hidden_layers"]),
        hidden=hidden,
        n_heads=heads,
        n_kv_heads=int(hc.get("num_key_value_heads") or heads),
        head_dim=head_dim,
        intermediate=int(hc["intermediate_size"]),
        vocab=vocab,
        rope_theta=theta,
        rms_eps=float(hc.get("rms_norm_eps", 1e-5)),
        max_position=max_pos,
        n_experts=int(hc.get("num_local_experts", 0) or 0),
        top_k_experts=int(hc.get("num_experts_per_tok", 0) or 0) if arch == "mixtral" else 0,
        rope_scaling=scaling,
        default_tp=1,
        checkpoint=os.path.abspath(path),
        bos_id=bos[0] if bos else -1,
        eos_ids=tuple(e for e in eos if 0 <= e < vocab),
        tie_embeddings=bool(hc.get("tie_word_embeddings", False)),
    )


def register_dir(root: str) -> List[str]:
    """Add every checkpoint under ``root`` (itself or its immediate subdirectories) to the
    catalog; returns the family names (directory basenames)."""
    dirs = [root] if is_checkpoint_dir(root) else sorted(
        d for d in glob.glob(os.path.join(root, "*")) if os.path.isdir(d) and is_checkpoint_dir(d))
    names = []
    for d in dirs:
        cfg = config_from_hf(d)
        old = FAMILIES.get(cfg.name)
        if old is not None and old.checkpoint != cfg.checkpoint:
            raise CheckpointError(f"checkpoint {d}: name {cfg.name!r} is already a catalog family")
        FAMILIES[cfg.name] = cfg
        names.append(cfg.name)
    return names


def _interleave(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """[I, H] x 2 -> [2I, H] with row 2i = gate_i, 2i + 1 = up_i (the engine's w_gu layout)."""
    return torch.stack([gate, up], 1).reshape(2 * gate.shape[0], gate.shape[1])


class HFCheckpoint:
    """Lazy tensor source over the safetensors shards of one checkpoint directory."""

    def __init__(self, path: str, cfg: ModelConfig):
        from safetensors import safe_open

        self.path = path
        self.cfg = cfg
        self._files = {}
        self._where: Dict[str, str] = {}
        files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
        if not files:
            raise CheckpointError(f"{path}: no *.safetensors files")
        for f in files:
            h = safe_open(f, framework="pt", device="cpu")
            self._files[f] = h
            for k in h.keys():
                self._where[k] = f

    def has(self, name: str) -> bool:
        return name in self._where

    def raw(self, name: str) -> torch.Tensor:
        f = self._where.get(name)
        if f is None:
            raise CheckpointError(f"{self.path}: tensor {name!r} missing")
        return self._files[f].get_tensor(name)

    def _first(self, *names: str) -> torch.Tensor:
        for n in names:
            if n in self._where:
                return self.raw(n)
        raise CheckpointError(f"{self.path}: none of {names} present")

    def get(self, key: str) -> torch.Tensor:
        """Full (unsharded) tensor for an engine weight key (see TransformerWeights._build)."""
        c = self.cfg
        if key == "embed":
            return self.raw("model.embed_tokens.weight")
        if key == "final_norm":
            return self.raw("model.norm.weight")
        if key == "lm_head":
            if self.has("lm_head.weight"):
                return self.raw("lm_head.weight")
            return self.raw("model.embed_tokens.weight")  # tied embeddings
        parts = key.split(".")
        i = int(parts[1])
        p = f"model.layers.{i}."
        leaf = parts[2]
        if leaf == "ln1":
            return self.raw(p + "input_layernorm.weight")
        if leaf == "ln2":
            return self.raw(p + "post_attention_layernorm.weight")
        if leaf == "w_qkv":
            if self.has(p + "self_attn.qkv_proj.weight"):
                return self.raw(p + "self_attn.qkv_proj.weight")
            return torch.cat([self.raw(p + f"self_attn.{x}_proj.weight") for x in "qkv"], 0)
        if leaf == "w_o":
            return self.raw(p + "self_attn.o_proj.weight")
        if leaf == "w_gu":
            if self.has(p + "mlp.gate_up_proj.weight"):
                gu = self.raw(p + "mlp.gate_up_proj.weight")
                return _interleave(gu[: c.intermediate], gu[c.intermediate:])
            return _interleave(self.raw(p + "mlp.gate_proj.weight"), self.raw(p + "mlp.up_proj.weight"))
        if leaf == "w_down":
            return self.raw(p + "mlp.down_proj.weight")
        if leaf == "w_router":
            return self._first(p + "block_sparse_moe.gate.weight", p + "mlp.gate.weight")
        if leaf == "experts":
            e, what = int(parts[3]), parts[4]
            hub = p + f"block_sparse_moe.experts.{e}."
            if what == "w_gu":
                if self.has(hub + "w1.weight"):
                    return _interleave(self.raw(hub + "w1.weight"), self.raw(hub + "w3.weight"))
                gu = self.raw(p + "mlp.experts.gate_up_proj")[e]
                return _interleave(gu[: c.intermediate], gu[c.intermediate:])
            if what == "w_down":
                if self.has(hub + "w2.weight"):
                    return self.raw(hub + "w2.weight")
                return self.raw(p + "mlp.experts.down_proj")[e]
        raise CheckpointError(f"unknown weight key {key!r}")
