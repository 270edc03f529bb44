"""Judge / consensus synthesis (reference ``internal/consensus/judge.go:12-105``).

* 0 responses → ``no responses to synthesize``;
* 1 response → passthrough: callback once with the content, judge model NOT called;
* otherwise render the judge prompt (text identical to the reference template) and make
  one streaming query to the judge; failures wrap as ``judge query failed: ...``.

The prompt is rendered as ``header + Σ block(response) + trailer`` so that a local judge
engine can prefill it incrementally as responses complete; the rendered
string is byte-identical to Go ``text/template`` output for the same inputs.
"""

from __future__ import annotations

from typing import List, Optional

from .context import Context
from .provider.base import Provider, Request, Response, StreamCallback

_HEADER = (
    "\n"
    "Role\n"
    "You are an expert synthesis judge and careful editor. Your job is to combine multiple AI model "
    "responses into one best-possible answer to the user.\n"
    "\n"
    "Inputs\n"
    "User's original prompt:\n"
)

_AFTER_PROMPT = "\n\nModel responses:\n"

_TRAILER = (
    "\n"
    "\n"
    "Task\n"
    "Produce ONE final answer that directly addresses the user's original prompt by synthesizing the "
    "model responses.\n"
    "\n"
    "Method\n"
    "1) Infer the user's intent and constraints from the original prompt (scope, tone, formatting, "
    "assumptions). Follow them.\n"
    "2) Extract the strongest points that are supported and/or repeated across responses.\n"
    "3) Resolve conflicts:\n"
    "   - Prefer statements that are more logically sound, more specific, and better justified.\n"
    "   - Prefer safer, broadly valid guidance over speculative or brittle claims.\n"
    "   - If uncertainty remains, choose the most defensible formulation and qualify it briefly.\n"
    "4) Fill gaps only when needed to make the answer complete and usable. Do not invent facts; do not "
    "add extraneous content.\n"
    "\n"
    "Output Requirements\n"
    "- Output ONLY the final synthesized answer (no preamble, no meta-commentary, no mention of models "
    "or “consensus”).\n"
    "- Do not quote or reference individual model responses.\n"
    "- Keep the answer coherent, non-redundant, and well-structured (use bullets/steps/headings if "
    "helpful).\n"
    "- Match formatting appropriate to the task (e.g., code blocks for code).\n"
)


def prompt_header(original_prompt: str) -> str:
    """Everything up to and including ``Model responses:\\n`` (before the first block)."""
    return _HEADER + original_prompt + _AFTER_PROMPT


def response_block(r: Response) -> str:
    """One ``{{range}}`` iteration (``judge.go:20-25``)."""
    return f"\n--- Model: {r.model} | Provider: {r.provider} ---\n{r.content}\n\n"


def prompt_trailer() -> str:
    return _TRAILER


def build_judge_prompt(original_prompt: str, responses: List[Response]) -> str:
    return prompt_header(original_prompt) + "".join(response_block(r) for r in responses) + _TRAILER


class JudgeError(Exception):
    pass


class Judge:
    def __init__(self, provider: Provider, model: str, request_template: Optional[Request] = None):
        self.provider = provider
        self.model = model
        self._tmpl = request_template

    def synthesize(self, ctx: Context, original_prompt: str, responses: List[Response]) -> str:
        return self.synthesize_stream(ctx, original_prompt, responses, None)

    def synthesize_stream(self, ctx: Context, original_prompt: str, responses: List[Response],
                          callback: Optional[StreamCallback]) -> str:
        if len(responses) == 0:
            raise JudgeError("no responses to synthesize")
        if len(responses) == 1:
            close = getattr(self.provider, "close_session", None)
            if close is not None:  # discard the partially prefilled judge KV
                close()
            if callback is not None:
                callback(responses[0].content)
            return responses[0].content
        prompt = build_judge_prompt(original_prompt, responses)
        req = Request(model=self.model, prompt=prompt)
        if self._tmpl is not None:
            import dataclasses

            req = dataclasses.replace(self._tmpl, model=self.model, prompt=prompt)
        try:
            finish = getattr(self.provider, "query_stream_session", None)
            if finish is not None:  # local judge: header + blocks already prefilled incrementally
                resp = finish(ctx, req, callback)
            else:
                resp = self.provider.query_stream(ctx, req, callback)
        except Exception as e:  # noqa: BLE001
            raise JudgeError(f"judge query failed: {e}") from e
        return resp.content
