"""Model catalog: which names the CLI accepts and which provider serves them.

Three kinds of names: local architectures (and ``--weights-dir`` checkpoints) served by the
MI355X engines, the reference's hosted model ids (served by ``provider/remote.py`` when their API
key is set), and the deterministic ``stub-*`` CPU family.

Reference: the closed ``knownModels`` map + ``createProvider`` (``cmd/llm-consensus/main.go:38-61,
417-438``) and the never-loaded ``models.json`` catalog produced by ``model-registry-sync``.
Here the catalog is the set of local architectures (``models/config.py``) plus a deterministic
CPU ``stub-*`` family (BASELINE config 1). A name is ``<family>[@<tag>]``: the tag selects a
distinct replica (its own random-init seed and engine instance), e.g. ``llama-3-8b@1``.
"""

from __future__ import annotations

import dataclasses
import json
import zlib
from typing import Dict, List, Optional

from .models.config import FAMILIES, ModelConfig

STUB_FAMILIES = ("stub",)
PROVIDER_LOCAL = "rocm"
PROVIDER_STUB = "stub"


class UnknownModel(Exception):
    pass


@dataclasses.dataclass(frozen=True)
class ModelSpec:
    name: str  # full CLI name
    family: str
    tag: str
    provider: str  # "rocm" | "stub"
    config: Optional[ModelConfig]

    @property
    def seed(self) -> int:
        """Deterministic weight seed per (family, tag)."""
        return zlib.crc32(f"{self.family}@{self.tag}".encode()) & 0x7FFFFFFF


def available_models() -> List[str]:
    from .provider.remote import KNOWN_REMOTE

    return sorted(FAMILIES) + sorted(KNOWN_REMOTE) + ["stub-<name>"]


def resolve(name: str) -> ModelSpec:
    from .provider.remote import KNOWN_REMOTE

    if name in KNOWN_REMOTE:  # the reference's hosted models (main.go:47-61), exact ids
        return ModelSpec(name, name, "", KNOWN_REMOTE[name], None)
    family, _, tag = name.partition("@")
    if family in FAMILIES:
        return ModelSpec(name, family, tag, PROVIDER_LOCAL, FAMILIES[family])
    if family.startswith("stub-") or family == "stub":
        return ModelSpec(name, family, tag, PROVIDER_STUB, None)
    raise UnknownModel(f'unknown model "{name}"; available models: [' + " ".join(available_models()) + "]")


def describe(name: str, tp: Optional[int] = None) -> Dict:
    """One catalog record (the ``model-registry-sync`` analogue)."""
    spec = resolve(name)
    if spec.config is None:
        return {"source": spec.provider, "id": name}
    c = spec.config
    tp = tp or c.default_tp
    return {
        "source": "checkpoint" if c.checkpoint else "local",
        "id": c.name,
        "arch": c.arch,
        "params": c.num_params(),
        "weight_bytes_bf16": c.weight_bytes(),
        "active_bytes_per_token_bf16": c.active_weight_bytes(),
        "kv_bytes_per_token_bf16": c.kv_bytes_per_token(),
        "context_length": c.max_position,
        "default_tp": c.default_tp,
        "per_rank_weight_bytes": c.weight_bytes() // tp,
        "layers": c.n_layers, "hidden": c.hidden, "heads": c.n_heads, "kv_heads": c.n_kv_heads,
        "head_dim": c.head_dim, "intermediate": c.intermediate, "vocab": c.vocab,
        "experts": c.n_experts, "top_k": c.top_k_experts,
        **({"path": c.checkpoint} if c.checkpoint else {}),
    }


def dump_catalog(indent: int = 2) -> str:
    recs = sorted((describe(n) for n in FAMILIES), key=lambda r: (r["source"], r["id"]))
    return json.dumps(recs, indent=indent) + "\n"
