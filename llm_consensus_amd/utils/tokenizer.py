"""Python face of the native synthetic tokenizer (``csrc/runtime/tokenizer.cpp``)."""

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
