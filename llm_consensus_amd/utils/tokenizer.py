"""Tokenizers: the native synthetic tokenizer (``csrc/runtime/tokenizer.cpp``) for
random-init architectures, and the checkpoint's own Hugging Face tokenizer (``tokenizer.json`` +
chat template) for ``--weights-dir`` models. Both expose encode / decode / ``encode_prompt`` (the
text a remote chat API would receive as one user message -> prompt ids) and an incremental
``stream_decoder`` for token streaming."""

from __future__ import annotations

import codecs
import functools
from typing import List, Sequence

from .native import runtime


class Tokenizer:
    def __init__(self, vocab_size: int):
        self._t = runtime().SyntheticTokenizer(int(vocab_size))
        self.vocab_size = int(vocab_size)
        self.bos_id = int(self._t.bos_id)
        self.eos_id = int(self._t.eos_id)

    def encode(self, text: str, add_bos: bool = False) -> List[int]:
        ids = self._t.encode(text.encode("utf-8", "surrogatepass"))
        return ([self.bos_id] + ids) if add_bos else ids

    def decode(self, ids: Sequence[int]) -> str:
        return self._t.decode_bytes(list(ids)).decode("utf-8", "replace")

    def decode_bytes(self, ids: Sequence[int]) -> bytes:
        return self._t.decode_bytes(list(ids))

    def piece_bytes(self, tok: int) -> bytes:
        return self._t.piece_bytes(int(tok))

    def stream_decoder(self) -> "StreamDecoder":
        return StreamDecoder(self)

    def encode_prompt(self, text: str) -> List[int]:
        return self.encode(text, add_bos=True)

    def prompt_prefix_ids(self, text: str) -> List[int]:
        """Ids of a prompt that starts with ``text`` (segment-stable: exact)."""
        return self.encode(text, add_bos=True)


class StreamDecoder:
    """Incremental detokenizer: byte tokens may split a UTF-8 sequence across chunks."""

    def __init__(self, tok: Tokenizer):
        self._tok = tok
        self._dec = codecs.getincrementaldecoder("utf-8")("replace")

    def push(self, ids: Sequence[int]) -> str:
        return self._dec.decode(b"".join(self._tok.piece_bytes(i) for i in ids))

    def flush(self) -> str:
        return self._dec.decode(b"", final=True)


@functools.lru_cache(maxsize=8)
def get_tokenizer(vocab_size: int) -> Tokenizer:
    return Tokenizer(vocab_size)


class HFTokenizer:
    """A checkpoint's tokenizer (``tokenizer.json``; chat template from ``tokenizer_config.json``),
    loaded from local files only."""

    def __init__(self, path: str, bos_id: int = -1, eos_ids=()):
        from transformers import AutoTokenizer

        self.path = path
        self._t = AutoTokenizer.from_pretrained(path, local_files_only=True)
        self.vocab_size = len(self._t)
        bid = self._t.bos_token_id if self._t.bos_token_id is not None else bos_id
        self.bos_id = int(bid) if bid is not None and bid >= 0 else -1
        self.eos_id = int(eos_ids[0]) if eos_ids else (self._t.eos_token_id if self._t.eos_token_id is not None else -1)
        self.has_chat_template = bool(getattr(self._t, "chat_template", None))

    def encode(self, text: str, add_bos: bool = False) -> List[int]:
        ids = list(self._t.encode(text, add_special_tokens=False))
        return ([self.bos_id] + ids) if add_bos and self.bos_id >= 0 else ids

    def encode_prompt(self, text: str) -> List[int]:
        if self.has_chat_template:
            out = self._t.apply_chat_template([{"role": "user", "content": text}], add_generation_prompt=True,
                                              tokenize=True)
            if isinstance(out, dict) or hasattr(out, "keys"):
                out = out["input_ids"]
            return [int(i) for i in out]
        return self.encode(text, add_bos=True)

    def prompt_prefix_ids(self, text: str) -> List[int]:
        """Best-effort ids of a prompt that starts with ``text``: the chat template's head (rendered
        around a sentinel message) followed by ``text``. Callers re-check against the full
        tokenization (query_stream_session)."""
        if not self.has_chat_template:
            return self.encode(text, add_bos=True)
        sentinel = "\x00llmc-sentinel\x00"
        rendered = self._t.apply_chat_template([{"role": "user", "content": sentinel}], add_generation_prompt=True,
                                               tokenize=False)
        head = rendered.split(sentinel)[0]
        return [int(i) for i in self._t.encode(head + text, add_special_tokens=False)]

    def decode(self, ids: Sequence[int]) -> str:
        return self._t.decode(list(ids), skip_special_tokens=True)

    def stream_decoder(self) -> "HFStreamDecoder":
        return HFStreamDecoder(self)


class HFStreamDecoder:
    """Incremental detokenization with a (prefix, read) window: text is emitted once the decode of
    the window grows and does not end in an incomplete UTF-8 sequence (U+FFFD)."""

    def __init__(self, tok: HFTokenizer):
        self._tok = tok
        self._ids: List[int] = []
        self._prefix = 0
        self._read = 0

    def _step(self, final: bool) -> str:
        before = self._tok.decode(self._ids[self._prefix:self._read])
        after = self._tok.decode(self._ids[self._prefix:])
        if len(after) > len(before) and (final or not after.endswith("\ufffd")):
            self._prefix, self._read = self._read, len(self._ids)
            return after[len(before):]
        return ""

    def push(self, ids: Sequence[int]) -> str:
        self._ids.extend(int(i) for i in ids)
        return self._step(False)

    def flush(self) -> str:
        return self._step(True)


_HF_CACHE: dict = {}


def tokenizer_for(cfg) -> "Tokenizer | HFTokenizer":
    """The tokenizer serving model config ``cfg``: the checkpoint's own when it ships one."""
    import os

    ck = getattr(cfg, "checkpoint", None)
    if ck and os.path.isfile(os.path.join(ck, "tokenizer.json")):
        t = _HF_CACHE.get(ck)
        if t is None:
            t = _HF_CACHE[ck] = HFTokenizer(ck, cfg.bos_id, cfg.eos_ids)
        return t
    return get_tokenizer(cfg.vocab)
