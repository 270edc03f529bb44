"""Version information (reference: ``cmd/llm-consensus/main.go:26-31, 287-296``).

The reference injects version/commit/date with ldflags; here the build step
(``__graft_entry__.build`` / ``build_ext.py``) may write ``_buildinfo.py``; otherwise
we fall back to "dev"/"none"/"unknown" exactly like the Go defaults.
"""

__version__ = "0.1.0"

version = "dev"
commit = "none"
date = "unknown"

try:  # written by the build step
    from ._buildinfo import version, commit, date  # type: ignore  # noqa: F401,F811
except Exception:  # pragma: no cover - absent in a source checkout
    pass


def get_version() -> str:
    """Mirror of ``getVersion`` (main.go:287-296): explicit version wins, else package version."""
    if version != "dev":
        return version
    return "dev"
