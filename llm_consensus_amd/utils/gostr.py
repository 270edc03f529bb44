"""Go string helpers whose exact semantics the contract depends on."""

from __future__ import annotations

import unicodedata

# unicode.IsSpace: '\t','\n','\v','\f','\r',' ', U+0085, U+00A0 and category Zs/Zl/Zp.
_LATIN1_SPACE = {"\t", "\n", "\v", "\f", "\r", " ", "\u0085", " "}


def is_go_space(ch: str) -> bool:
    if ord(ch) < 0x100:
        return ch in _LATIN1_SPACE
    return unicodedata.category(ch) in ("Zs", "Zl", "Zp")


def trim_space(s: str) -> str:
    """``strings.TrimSpace``."""
    i, j = 0, len(s)
    while i < j and is_go_space(s[i]):
        i += 1
    while j > i and is_go_space(s[j - 1]):
        j -= 1
    return s[i:j]


def truncate_bytes(s: str, max_len: int) -> str:
    """``ui.truncate`` (internal/ui/ui.go:251-259): newlines → spaces, TrimSpace, then cut on
    BYTES to ``max_len-1`` + "…" (so a multi-byte rune can be split; the split bytes are kept as
    surrogate escapes and written back raw by the UI writer)."""
    s = trim_space(s.replace("\n", " "))
    b = s.encode("utf-8", "surrogateescape")
    if len(b) > max_len:
        return b[: max_len - 1].decode("utf-8", "surrogateescape") + "…"
    return s


def go_fmt_list(items) -> str:
    """``fmt.Sprintf("%v", []string{...})``."""
    return "[" + " ".join(items) + "]"
