"""Packaging for llm-consensus-amd (the reference ships a GoReleaser config, ``.goreleaser.yaml``).

The HIP extension and host runtime are compiled by ``__graft_entry__.build()`` (hipcc for gfx950)
into ``llm_consensus_amd/_lib/`` first; the wheel only carries the built ``.so`` files, so it is
platform-specific to ROCm 7 / gfx950. ``scripts/release.sh`` stamps version/commit/date and runs
both steps.
"""

import re
from pathlib import Path

from setuptools import Distribution, find_packages, setup


class _BinaryDistribution(Distribution):
    """Carries prebuilt gfx950 extension modules: tag the wheel for this platform/ABI."""

    def has_ext_modules(self):
        return True

_here = Path(__file__).parent
_ver = re.search(r'^__version__ = "([^"]+)"', (_here / "llm_consensus_amd" / "version.py").read_text(), re.M)

setup(
    name="llm-consensus-amd",
    version=_ver.group(1),
    description="Multi-model consensus engine for AMD Instinct MI355X (gfx950): "
                "llm-consensus CLI on local HIP/CDNA4 inference",
    long_description=(_here / "README.md").read_text(encoding="utf-8"),
    long_description_content_type="text/markdown",
    python_requires=">=3.10",
    packages=find_packages(include=["llm_consensus_amd", "llm_consensus_amd.*"]),
    package_data={"llm_consensus_amd": ["_lib/*.so"]},
    install_requires=["torch", "numpy"],
    extras_require={"checkpoints": ["safetensors", "transformers", "tokenizers", "jinja2"],
                    "remote": ["httpx"]},
    entry_points={"console_scripts": [
        "llm-consensus = llm_consensus_amd.cli:main",
        "llm-consensus-server = llm_consensus_amd.server:main",
        "model-registry-sync = llm_consensus_amd.registry_sync:main",
    ]},
    distclass=_BinaryDistribution,
    zip_safe=False,
)
