"""``model-registry-sync``: snapshot of the models this node can serve, as a sorted JSON array.

Reference: ``cmd/model-registry-sync/main.go`` lists the remote catalogs of OpenAI
(``GET /v1/models``) and OpenRouter (``GET /api/v1/models``) into ``[]ModelRecord`` sorted by
(source, id), prints to stdout or ``-out``, and reports per-source failures as warnings at the end
without failing the run (main.go:63-127). On an offline MI355X node the "remote catalogs" become
local sources, kept with the same flag style, record shape and failure semantics:

* ``local``       — the built-in random-init architectures (``models/config.py``);
* ``checkpoint``  — Hugging Face checkpoint directories (``-weights-dir``, ``$LLMC_WEIGHTS_DIR``);
* ``hf-cache``    — snapshots in the Hugging Face hub cache (``$HF_HOME``/hub, read-only scan);
* ``openai`` / ``openrouter`` — the reference's own remote sources, same requests and records
  (``GET {base}/models``; OpenAI needs ``OPENAI_API_KEY``, OpenRouter sends ``OPENROUTER_API_KEY``
  when set; main.go:129-213), base URLs overridable (``OPENAI_BASE_URL``, ``OPENROUTER_BASE_URL``).

Each record: ``source``, ``id``, ``name``, ``context_length`` (the reference's fields, pricing
dropped: local inference has none) plus what placement needs (params, bf16 weight bytes, KV bytes
per token, default TP); ``-raw`` adds the model's full config.
"""

from __future__ import annotations

import dataclasses
import glob
import json
import os
import sys
import time
from typing import List, Optional, TextIO

from .flags import FlagSet, parse_or_exit


def _record(source: str, rid: str, cfg, raw: bool) -> dict:
    rec = {"source": source, "id": rid, "name": cfg.name, "context_length": cfg.max_position,
           "arch": cfg.arch, "params": cfg.num_params(), "weight_bytes_bf16": cfg.weight_bytes(),
           "kv_bytes_per_token_bf16": cfg.kv_bytes_per_token(), "default_tp": cfg.default_tp}
    if cfg.checkpoint:
        rec["path"] = cfg.checkpoint
    if raw:
        d = dataclasses.asdict(cfg)
        d["eos_ids"] = list(d.get("eos_ids") or ())
        rec["raw"] = d
    return rec


def local_records(raw: bool) -> List[dict]:
    from .models.config import FAMILIES

    return [_record("local", n, c, raw) for n, c in FAMILIES.items() if not c.checkpoint]


def checkpoint_records(dirs: List[str], raw: bool, deadline: float) -> List[dict]:
    from .models.checkpoint import config_from_hf, is_checkpoint_dir

    out = []
    for root in dirs:
        if not os.path.isdir(root):
            raise FileNotFoundError(f"{root}: no such directory")
        cands = [root] if is_checkpoint_dir(root) else sorted(glob.glob(os.path.join(root, "*")))
        for d in cands:
            if time.monotonic() > deadline:
                raise TimeoutError("scan timed out")
            if os.path.isdir(d) and is_checkpoint_dir(d):
                cfg = config_from_hf(d)
                out.append(_record("checkpoint", cfg.name, cfg, raw))
    return out


def hf_cache_records(raw: bool, deadline: float) -> List[dict]:
    from .models.checkpoint import CheckpointError, config_from_hf, is_checkpoint_dir

    home = os.environ.get("HF_HOME") or os.path.join(os.path.expanduser("~"), ".cache", "huggingface")
    hub = os.environ.get("HF_HUB_CACHE") or os.path.join(home, "hub")
    out = []
    for repo in sorted(glob.glob(os.path.join(hub, "models--*"))):
        if time.monotonic() > deadline:
            raise TimeoutError("scan timed out")
        rid = os.path.basename(repo)[len("models--"):].replace("--", "/")
        for snap in sorted(glob.glob(os.path.join(repo, "snapshots", "*"))):
            if is_checkpoint_dir(snap):
                try:
                    cfg = config_from_hf(snap, name=rid)
                except CheckpointError:
                    continue  # an architecture this engine does not serve
                out.append(_record("hf-cache", rid, cfg, raw))
                break
    return out


def _get_json(url: str, headers: dict, timeout: float):
    import httpx

    r = httpx.get(url, headers=headers, timeout=timeout)
    if r.status_code < 200 or r.status_code >= 300:
        body = r.text
        raise RuntimeError(f"http {r.status_code}: {body[:600] + ('…' if len(body) > 600 else '')}")
    try:
        return r.json()
    except ValueError as e:
        raise RuntimeError(f"unmarshal: {e}; body={r.text[:600]}") from None


def openai_records(raw: bool, timeout: float) -> List[dict]:
    key = os.environ.get("OPENAI_API_KEY", "").strip()
    if not key:
        raise RuntimeError("OPENAI_API_KEY not set")
    base = os.environ.get("OPENAI_BASE_URL", "https://api.openai.com/v1").rstrip("/")
    data = _get_json(f"{base}/models", {"Authorization": f"Bearer {key}"}, timeout)
    out = []
    for m in data.get("data") or []:
        rec = {"source": "openai", "id": m.get("id", "")}
        if raw:
            rec["raw"] = m
        out.append(rec)
    return out


def openrouter_records(raw: bool, timeout: float) -> List[dict]:
    base = os.environ.get("OPENROUTER_BASE_URL", "https://openrouter.ai/api/v1").rstrip("/")
    key = os.environ.get("OPENROUTER_API_KEY", "").strip()
    data = _get_json(f"{base}/models", {"Authorization": f"Bearer {key}"} if key else {}, timeout)
    out = []
    for m in data.get("data") or []:
        rec = {"source": "openrouter", "id": m.get("id", "")}
        if m.get("name"):
            rec["name"] = m["name"]
        if m.get("context_length"):
            rec["context_length"] = m["context_length"]
        rec["pricing"] = {k: (m.get("pricing") or {}).get(k, "") for k in ("prompt", "completion", "request", "image")}
        if raw:
            rec["raw"] = m
        out.append(rec)
    return out


def main(argv: Optional[List[str]] = None, stdout: TextIO = sys.stdout, stderr: TextIO = sys.stderr) -> int:
    fs = FlagSet("model-registry-sync")
    fs.add("out", "string", "", "output file path (defaults to stdout)")
    fs.add("raw", "bool", False, "include raw model configs in output (debugging)")
    fs.add("local", "bool", True, "list the built-in architectures")
    fs.add("weights-dir", "string", "", "comma-separated checkpoint dirs to scan (default $LLMC_WEIGHTS_DIR)")
    fs.add("hf-cache", "bool", True, "scan the Hugging Face hub cache")
    fs.add("openai", "bool", True, "fetch OpenAI models (requires OPENAI_API_KEY)")
    fs.add("openrouter", "bool", True, "fetch OpenRouter models (uses OPENROUTER_API_KEY if set)")
    fs.add("timeout", "int", 20, "HTTP / scan timeout in seconds")
    v, _ = parse_or_exit(fs, list(sys.argv[1:] if argv is None else argv), stderr)
    deadline = time.monotonic() + max(1, v["timeout"])
    all_recs: List[dict] = []
    errs: List[str] = []
    if v["local"]:
        all_recs += local_records(v["raw"])
    wd = v["weights_dir"] or os.environ.get("LLMC_WEIGHTS_DIR", "")
    dirs = [d.strip() for d in wd.split(",") if d.strip()]
    if dirs:
        try:
            all_recs += checkpoint_records(dirs, v["raw"], deadline)
        except Exception as e:  # noqa: BLE001 - a failed source is a warning (main.go:120-126)
            errs.append(f"checkpoint: {e}")
    if v["hf_cache"]:
        try:
            all_recs += hf_cache_records(v["raw"], deadline)
        except Exception as e:  # noqa: BLE001
            errs.append(f"hf-cache: {e}")
    for flag, name, fn in (("openai", "openai", openai_records), ("openrouter", "openrouter", openrouter_records)):
        if v[flag]:
            try:
                all_recs += fn(v["raw"], float(v["timeout"]))
            except Exception as e:  # noqa: BLE001
                errs.append(f"{name}: {e}")
    all_recs.sort(key=lambda r: (r["source"], r["id"]))
    payload = json.dumps(all_recs, indent=2)
    if v["out"] == "":
        stdout.write(payload + "\n")
    else:
        try:
            with open(v["out"], "w", encoding="utf-8") as f:
                f.write(payload)
        except OSError as e:
            stderr.write(f"ERROR: {e}\n")
            return 1
    if errs:
        stderr.write("\nWARN: some sources failed:\n")
        for e in errs:
            stderr.write(f" - {e}\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
