"""Terminal UI on stderr (reference ``internal/ui/ui.go``).

Same state machine (pending → running → streaming → complete/failed), the same 100 ms
re-render of an N+2-line block with ANSI cursor-up/clear, the same byte strings.  The one
behavioural improvement: the token count shown is the EXACT count of generated tokens when the
provider reports it (local engines do), falling back to the reference's chars/4 estimate.
The reference's unlocked read of ``rendered`` in ``Stop`` is not reproduced:
all state, including ``rendered``, is read under the lock.
"""

from __future__ import annotations

import enum
import os
import sys
import threading
import time
from typing import Dict, List, Optional, TextIO

from .utils.gostr import truncate_bytes

RESET = "\033[0m"
BOLD = "\033[1m"
DIM = "\033[2m"
GREEN = "\033[32m"
YELLOW = "\033[33m"
BLUE = "\033[34m"
MAGENTA = "\033[35m"
CYAN = "\033[36m"
RED = "\033[31m"
BOLD_GREEN = "\033[1;32m"
BOLD_YELLOW = "\033[1;33m"
BOLD_BLUE = "\033[1;34m"
BOLD_CYAN = "\033[1;36m"

_SPINNER = ["⠋", "⠙", "⠹", "⠸", "⠼", "⠴", "⠦", "⠧", "⠇", "⠏"]


def _write(w: TextIO, s: str) -> None:
    buf = getattr(w, "buffer", None)
    if buf is not None:
        buf.write(s.encode("utf-8", "surrogateescape"))
        buf.flush()
    else:
        w.write(s)
    try:
        w.flush()
    except Exception:  # noqa: BLE001
        pass


class Status(enum.IntEnum):
    PENDING = 0
    RUNNING = 1
    STREAMING = 2
    COMPLETE = 3
    FAILED = 4


class ModelState:
    __slots__ = ("model", "status", "start", "end", "error", "char_count", "token_est", "last_chunk", "exact_tokens")

    def __init__(self, model: str):
        self.model = model
        self.status = Status.PENDING
        self.start = 0.0
        self.end = 0.0
        self.error: Optional[BaseException] = None
        self.char_count = 0
        self.token_est = 0
        self.last_chunk = ""
        self.exact_tokens: Optional[int] = None


def spinner(t: Optional[float] = None) -> str:
    t = time.time() if t is None else t
    return _SPINNER[int(t * 1000) // 100 % len(_SPINNER)]


class Progress:
    def __init__(self, w: TextIO, models: List[str], quiet: bool):
        self._lock = threading.Lock()
        self._w = w
        self._order = list(models)
        self._models: Dict[str, ModelState] = {m: ModelState(m) for m in models}
        self._start = time.monotonic()
        self._quiet = quiet
        self._rendered = False
        self._done = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def start(self) -> None:
        if self._quiet:
            return

        def loop() -> None:
            while not self._done.wait(0.1):
                self.render()

        self._thread = threading.Thread(target=loop, daemon=True, name="ui-progress")
        self._thread.start()
        self.render()

    def stop(self) -> None:
        if self._quiet:
            return
        self._done.set()
        if self._thread is not None:
            self._thread.join()
        with self._lock:
            if self._rendered:
                self._clear_lines(len(self._order) + 2)

    # -- state transitions (ui.go:123-168) ---------------------------------------------------
    def model_started(self, model: str) -> None:
        with self._lock:
            st = self._models.get(model)
            if st:
                st.status = Status.RUNNING
                st.start = time.monotonic()

    def model_streaming(self, model: str, chunk: str, tokens: Optional[int] = None) -> None:
        with self._lock:
            st = self._models.get(model)
            if st:
                st.status = Status.STREAMING
                st.char_count += len(chunk.encode("utf-8", "surrogateescape"))
                if tokens is not None:
                    st.exact_tokens = (st.exact_tokens or 0) + tokens
                st.token_est = st.exact_tokens if st.exact_tokens is not None else st.char_count // 4
                st.last_chunk = truncate_bytes(chunk, 30)

    def model_tokens(self, model: str, n: int) -> None:
        """Exact generated-token count from a local engine (replaces the chars/4 estimate)."""
        with self._lock:
            st = self._models.get(model)
            if st:
                st.exact_tokens = (st.exact_tokens or 0) + n
                st.token_est = st.exact_tokens

    def model_completed(self, model: str) -> None:
        with self._lock:
            st = self._models.get(model)
            if st:
                st.status = Status.COMPLETE
                st.end = time.monotonic()

    def model_failed(self, model: str, err: BaseException) -> None:
        with self._lock:
            st = self._models.get(model)
            if st:
                st.status = Status.FAILED
                st.end = time.monotonic()
                st.error = err

    # -- rendering (ui.go:170-249) -----------------------------------------------------------
    def render(self) -> None:
        with self._lock:
            out = []
            if self._rendered:
                out.append("\033[A\033[K" * (len(self._order) + 2))
            self._rendered = True
            elapsed = time.monotonic() - self._start
            out.append(f"{BOLD_CYAN}⚡ Querying {len(self._order)} models{RESET} {DIM}({elapsed:.1f}s){RESET}\n")
            for m in self._order:
                out.append(self._model_line(self._models[m]))
            out.append("\n")
            _write(self._w, "".join(out))

    def _model_line(self, st: ModelState) -> str:
        now = time.monotonic()
        if st.status == Status.PENDING:
            icon, color, status = "○", DIM, "pending"
        elif st.status == Status.RUNNING:
            icon, color, status = spinner(), YELLOW, f"connecting... {now - st.start:.1f}s"
        elif st.status == Status.STREAMING:
            icon, color, status = spinner(), CYAN, f"streaming ~{st.token_est} tokens {now - st.start:.1f}s"
        elif st.status == Status.COMPLETE:
            icon, color, status = "✓", GREEN, f"done ~{st.token_est} tokens in {st.end - st.start:.1f}s"
        else:
            icon, color, status = "✗", RED, f"failed: {st.error}"
        name = truncate_bytes(st.model, 25)
        pad = " " * max(0, 25 - len(name))  # Go %-25s pads by runes
        return f"  {color}{icon}{RESET} {name}{pad} {color}{status}{RESET}\n"

    def _clear_lines(self, n: int) -> None:
        _write(self._w, "\033[A\033[K" * n)

    # Test hook
    def state(self, model: str) -> ModelState:
        return self._models[model]


def print_header(w: TextIO, prompt: str) -> None:
    _write(w, f"\n{BOLD_CYAN}╭─ LLM Consensus ─╮{RESET}\n"
              f"{CYAN}│{RESET} Prompt: {DIM}{truncate_bytes(prompt, 60)}{RESET}\n"
              f"{CYAN}╰─────────────────╯{RESET}\n\n")


def print_phase(w: TextIO, phase: str) -> None:
    _write(w, f"{BOLD_YELLOW}▸ {phase}{RESET}\n")


def print_success(w: TextIO, msg: str) -> None:
    _write(w, f"{GREEN}✓ {msg}{RESET}\n")


def print_error(w: TextIO, msg: str) -> None:
    _write(w, f"{RED}✗ {msg}{RESET}\n")


def print_model_response(w: TextIO, model: str, provider: str, content: str, latency_s: float) -> None:
    out = [f"\n{BLUE}┌─ {model} ({provider}) [{latency_s:.1f}s] ─┐{RESET}\n"]
    for line in content.split("\n"):
        out.append(f"{BLUE}│{RESET} {line}\n")
    out.append(f"{BLUE}└─────────────────────────┘{RESET}\n")
    _write(w, "".join(out))


def print_consensus(w: TextIO, consensus: str) -> None:
    out = [f"\n{BOLD_GREEN}╔═══ CONSENSUS ═══╗{RESET}\n"]
    for line in consensus.split("\n"):
        out.append(f"{GREEN}║{RESET} {line}\n")
    out.append(f"{GREEN}╚═════════════════╝{RESET}\n")
    _write(w, "".join(out))


def print_summary(w: TextIO, total: int, ok: int, failed: int, total_s: float) -> None:
    _write(w, f"\n{DIM}─── Summary ───{RESET}\n"
              f"Models queried: {total} ({GREEN}{ok} succeeded{RESET}, {RED}{failed} failed{RESET})\n"
              f"Total time: {total_s:.1f}s\n")


def is_terminal(f) -> bool:
    """``IsTerminal``: the file is a character device (ui.go:319-322)."""
    try:
        import stat

        return stat.S_ISCHR(os.fstat(f.fileno()).st_mode)
    except Exception:  # noqa: BLE001
        return False


def stderr() -> TextIO:
    return sys.stderr
