"""Result schema + Go-compatible JSON (reference ``internal/output/output.go:7-15``,
``internal/provider/provider.go:30-35``, encoder setup ``cmd/llm-consensus/main.go:227-228``).

Byte-for-byte fidelity with ``json.NewEncoder(w).SetIndent("", "  ").Encode(out)``:
* key order ``prompt, responses, consensus, judge, warnings, failed_models``;
  response keys ``model, content, provider, latency_ms``;
* ``warnings`` / ``failed_models`` omitted when empty (``omitempty``);
* HTML-escaping of ``< > &``, U+2028/2029, invalid UTF-8 → U+FFFD (native
  ``go_json_string`` in ``csrc/runtime/gojson.cpp``);
* two-space indent, trailing newline.
Deliberate deviation: ``latency_ms`` is milliseconds (the Go binary writes ns).
"""

from __future__ import annotations

import dataclasses
from typing import List, Optional

from .provider.base import Response
from .utils.native import runtime


@dataclasses.dataclass
class Result:
    prompt: str
    responses: List[Response]
    consensus: str
    judge: str
    warnings: Optional[List[str]] = None
    failed_models: Optional[List[str]] = None


def go_string(s: str) -> str:
    return runtime().go_json_string(s.encode("utf-8", "surrogatepass")).decode("utf-8")


def _response_lines(r: Response, ind: str) -> List[str]:
    i2 = ind + "  "
    return [
        ind + "{",
        f'{i2}"model": {go_string(r.model)},',
        f'{i2}"content": {go_string(r.content)},',
        f'{i2}"provider": {go_string(r.provider)},',
        f'{i2}"latency_ms": {int(r.latency_ms)}',
        ind + "}",
    ]


def _str_array(items: Optional[List[str]], ind: str) -> str:
    if items is None:
        return "null"
    if len(items) == 0:
        return "[]"
    inner = ",\n".join(ind + "  " + go_string(x) for x in items)
    return "[\n" + inner + "\n" + ind + "]"


def encode_result(res: Result) -> str:
    """Return the exact text Go's indented ``json.Encoder`` writes for ``output.Result``."""
    fields = [f'  "prompt": {go_string(res.prompt)}']
    if res.responses is None:
        fields.append('  "responses": null')
    elif len(res.responses) == 0:
        fields.append('  "responses": []')
    else:
        blocks = []
        for r in res.responses:
            blocks.append("\n".join(_response_lines(r, "    ")))
        fields.append('  "responses": [\n' + ",\n".join(blocks) + "\n  ]")
    fields.append(f'  "consensus": {go_string(res.consensus)}')
    fields.append(f'  "judge": {go_string(res.judge)}')
    if res.warnings:
        fields.append('  "warnings": ' + _str_array(res.warnings, "  "))
    if res.failed_models:
        fields.append('  "failed_models": ' + _str_array(res.failed_models, "  "))
    return "{\n" + ",\n".join(fields) + "\n}\n"
