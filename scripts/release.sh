#!/bin/bash
# Release build (the reference's GoReleaser + ldflags -X main.version/commit/date analogue):
# stamps version/commit/date into llm_consensus_amd/_buildinfo.py, builds every native module
# for gfx950 in-tree, and builds a wheel that carries the .so files.
# usage: bash scripts/release.sh [version]   (default: git describe)
set -euo pipefail
cd "$(dirname "$0")/.."
ver=${1:-$(git describe --tags --always 2>/dev/null || echo dev)}
commit=$(git rev-parse --short HEAD 2>/dev/null || echo none)
date=$(date -u +%Y-%m-%dT%H:%M:%SZ)
cat > llm_consensus_amd/_buildinfo.py <<PY
version = "${ver}"
commit = "${commit}"
date = "${date}"
PY
python -c "import __graft_entry__ as g; g.build()"
python -m pip wheel --no-deps --no-build-isolation -w dist . >/dev/null
echo "built dist/ for ${ver} (${commit}, ${date})"
