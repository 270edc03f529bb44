"""Model-name → Provider registry (reference ``internal/provider/registry.go:8-53``).

Populated once at bootstrap and then only read; a lock keeps ``register`` safe if a caller
does register concurrently (the reference uses an RWMutex).
"""

from __future__ import annotations

import threading
from typing import Dict, List

from .base import Provider


class UnknownModelError(KeyError):
    def __str__(self) -> str:  # KeyError would repr-quote the message
        return self.args[0]


class Registry:
    def __init__(self) -> None:
        self._lock = threading.Lock()
        self._providers: Dict[str, Provider] = {}

    def register(self, model: str, provider: Provider) -> None:
        with self._lock:
            self._providers[model] = provider

    def get(self, model: str) -> Provider:
        with self._lock:
            p = self._providers.get(model)
        if p is None:
            raise UnknownModelError(f"unknown model: {model}")
        return p

    def models(self) -> List[str]:
        with self._lock:
            return list(self._providers)

    def close(self) -> None:
        """Release backend resources (engines/workers) of every provider that has any."""
        with self._lock:
            provs = list(self._providers.values())
        seen = set()
        for p in provs:
            if id(p) in seen:
                continue
            seen.add(id(p))
            close = getattr(p, "close", None)
            if close is not None:
                close()
