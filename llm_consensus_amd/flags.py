"""Go ``flag`` package semantics (reference ``cmd/llm-consensus/main.go:298-361``).

Reproduced: ``-x`` ≡ ``--x``; ``-x=v`` and ``-x v``; parsing stops at the first non-flag
argument (or after ``--``), so flags after the prompt become prompt text; bool flags take no
separate value; ``-h``/``-help`` print usage and exit 0; unknown flags, missing arguments and
bad values print the error + usage to stderr and exit 2; integers accept Go's base prefixes.
"""

from __future__ import annotations

import dataclasses
import sys
from typing import Any, Callable, Dict, List, Optional, TextIO, Tuple


class FlagError(Exception):
    pass


class HelpRequested(Exception):
    pass


@dataclasses.dataclass
class Flag:
    name: str
    kind: str  # "string" | "int" | "bool" | "float"
    default: Any
    usage: str
    dest: str


def _parse_bool(s: str) -> bool:
    if s in ("1", "t", "T", "TRUE", "true", "True"):
        return True
    if s in ("0", "f", "F", "FALSE", "false", "False"):
        return False
    raise ValueError("parse error")


def _parse_int(s: str) -> int:
    # strconv.ParseInt(s, 0, 64): optional sign, 0x/0o/0b/0 prefixes, '_' only with a prefix.
    t = s
    sign = 1
    if t[:1] in ("+", "-"):
        sign = -1 if t[0] == "-" else 1
        t = t[1:]
    if not t:
        raise ValueError("parse error")
    base = 10
    low = t.lower()
    if low.startswith("0x"):
        base, t = 16, t[2:]
    elif low.startswith("0o"):
        base, t = 8, t[2:]
    elif low.startswith("0b"):
        base, t = 2, t[2:]
    elif len(t) > 1 and t[0] == "0":
        base, t = 8, t[1:]
    if base == 10 and "_" in t:
        raise ValueError("parse error")
    if not t or t.startswith("_") or t.endswith("_") or "__" in t:
        raise ValueError("parse error")
    try:
        v = sign * int(t.replace("_", ""), base)
    except ValueError:
        raise ValueError("parse error") from None
    if not -(2**63) <= v < 2**63:
        raise ValueError("value out of range")
    return v


def _parse_float(s: str) -> float:
    try:
        return float(s.replace("_", ""))
    except ValueError:
        raise ValueError("parse error") from None


_PARSERS: Dict[str, Callable[[str], Any]] = {"int": _parse_int, "bool": _parse_bool, "float": _parse_float, "string": str}


class FlagSet:
    def __init__(self, prog: str):
        self.prog = prog
        self._flags: Dict[str, Flag] = {}

    def add(self, name: str, kind: str, default: Any, usage: str, dest: Optional[str] = None) -> None:
        self._flags[name] = Flag(name, kind, default, usage, dest or name.replace("-", "_"))

    def usage(self) -> str:
        out = [f"Usage of {self.prog}:\n"]
        for name in sorted(self._flags):
            f = self._flags[name]
            line = f"  -{name}"
            tname = "" if f.kind == "bool" else ("value" if f.kind == "float" else f.kind)
            if f.kind == "float":
                tname = "float"
            if tname:
                line += " " + tname
            line += "\t" if len(line) <= 4 else "\n    \t"
            line += f.usage.replace("\n", "\n    \t")
            if f.kind == "string" and f.default != "":
                line += f' (default "{f.default}")'
            elif f.kind == "int" and f.default != 0:
                line += f" (default {f.default})"
            elif f.kind == "float" and f.default != 0:
                line += f" (default {_go_float(f.default)})"
            elif f.kind == "bool" and f.default:
                line += " (default true)"
            out.append(line + "\n")
        return "".join(out)

    def parse(self, argv: List[str]) -> Tuple[Dict[str, Any], List[str]]:
        values: Dict[str, Any] = {f.dest: f.default for f in self._flags.values()}
        args = list(argv)
        while args:
            s = args[0]
            if len(s) < 2 or s[0] != "-":
                break
            num_minuses = 1
            if s[1] == "-":
                num_minuses = 2
                if len(s) == 2:  # "--" terminates flags
                    args.pop(0)
                    break
            name = s[num_minuses:]
            if len(name) == 0 or name[0] == "-" or name[0] == "=":
                raise FlagError(f"bad flag syntax: {s}")
            args.pop(0)
            has_value = False
            value = ""
            if "=" in name[1:]:
                i = name.index("=", 1)
                value = name[i + 1:]
                has_value = True
                name = name[:i]
            f = self._flags.get(name)
            if f is None:
                if name in ("help", "h"):
                    raise HelpRequested()
                raise FlagError(f"flag provided but not defined: -{name}")
            if f.kind == "bool":
                if has_value:
                    try:
                        values[f.dest] = _parse_bool(value)
                    except ValueError as e:
                        raise FlagError(f'invalid boolean value "{value}" for -{name}: {e}') from None
                else:
                    values[f.dest] = True
                continue
            if not has_value:
                if not args:
                    raise FlagError(f"flag needs an argument: -{name}")
                value = args.pop(0)
            try:
                values[f.dest] = _PARSERS[f.kind](value)
            except ValueError as e:
                raise FlagError(f'invalid value "{value}" for flag -{name}: {e}') from None
        return values, args


def _go_float(v: float) -> str:
    r = repr(float(v))
    return r[:-2] if r.endswith(".0") else r


def parse_or_exit(fs: FlagSet, argv: List[str], err: TextIO = sys.stderr) -> Tuple[Dict[str, Any], List[str]]:
    """``flag.Parse`` with ``ExitOnError``: exit 0 on -h, exit 2 on errors (usage printed)."""
    try:
        return fs.parse(argv)
    except HelpRequested:
        err.write(fs.usage())
        err.flush()
        raise SystemExit(0)
    except FlagError as e:
        err.write(f"{e}\n{fs.usage()}")
        err.flush()
        raise SystemExit(2)
