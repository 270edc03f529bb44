"""``llm-consensus`` entry point (reference composition root ``cmd/llm-consensus/main.go:76-438``).

Flow, strings, output routing and exit codes match the reference:
parse flags → prompt (args > --file > piped stdin) → registry bootstrap (every ``--models``
entry and the judge must resolve, main.go:395-415) → fan-out → judge → persist/print.
"Providers" are local engines on the node's GPUs (``provider/local.py``) or the CPU stub.

Extra engine flags (no reference counterpart): ``--max-tokens``,
``--temperature``, ``--top-p``, ``--top-k``, ``--seed``, ``--gpus``, ``--trace``,
``--list-models``, ``--weights-dir`` (Hugging Face checkpoints as extra local model families),
``--placement`` (pin models / TP groups to GPUs).
"""

from __future__ import annotations

import dataclasses
import os
import secrets
import signal
import stat
import sys
import time
from typing import List, Optional, TextIO

from . import ui
from .catalog import PROVIDER_LOCAL, PROVIDER_STUB, UnknownModel, dump_catalog, resolve
from .consensus import Judge, prompt_header, response_block
from .context import Context
from .flags import FlagSet, parse_or_exit
from .output import Result, encode_result
from .provider.base import Request
from .provider.registry import Registry
from .runner import Callbacks, Runner
from .utils.gostr import trim_space
from .version import commit, date, get_version

DEFAULT_JUDGE = "llama-3-8b@judge"
PROG = "llm-consensus"


class CLIError(Exception):
    pass


@dataclasses.dataclass
class Config:
    models: List[str]
    judge: str
    file: str
    output: str
    data_dir: str
    timeout: float
    prompt: str
    quiet: bool
    json: bool
    no_save: bool
    max_tokens: int
    temperature: float
    top_p: float
    top_k: int
    seed: int
    gpus: str
    trace: bool
    placement: str = ""
    judge_tp: int = 0
    server: str = ""
    judge_explicit: bool = True


def make_flagset() -> FlagSet:
    fs = FlagSet(PROG)
    fs.add("models", "string", "", "Comma-separated list of models to query (required)")
    fs.add("judge", "string", DEFAULT_JUDGE, "Model to use for consensus synthesis")
    fs.add("file", "string", "", "Read prompt from file")
    fs.add("output", "string", "", "Write JSON output to specific file (overrides auto-save)")
    fs.add("data-dir", "string", "data", "Directory for auto-saved runs")
    fs.add("timeout", "int", 120, "Per-model timeout in seconds")
    fs.add("quiet", "bool", False, "Suppress progress output")
    fs.add("q", "bool", False, "Suppress progress output (shorthand)", dest="quiet")
    fs.add("json", "bool", False, "Output JSON to stdout (no interactive display, no auto-save)")
    fs.add("no-save", "bool", False, "Don't auto-save results to data directory")
    fs.add("version", "bool", False, "Print version information and exit")
    # engine flags
    fs.add("max-tokens", "int", 0, "Max generated tokens per model (0 = engine default: 4096 local, 24 stub)")
    fs.add("temperature", "float", 1.0, "Sampling temperature (0 = greedy)")
    fs.add("top-p", "float", 1.0, "Nucleus sampling mass")
    fs.add("top-k", "int", 0, "Top-k sampling (0 = off)")
    fs.add("seed", "int", 0, "Sampling seed (0 = derived from the model name)")
    fs.add("gpus", "string", "", "Comma-separated GPU ids to place models on (default: all visible)")
    fs.add("trace", "bool", False, "Write a Chrome trace of engine spans to the run directory")
    fs.add("placement", "string", "",
           "Pin models to GPUs: model=gpu[+gpu...],... ('+' = tensor-parallel group); the rest are placed automatically")
    fs.add("judge-tp", "int", 0,
           "Run a local judge tensor-parallel over the first N GPUs, beside the responders (0 = placed by the solver)")
    fs.add("server", "string", "",
           "Send the run to a running llm-consensus server (URL) instead of starting engines ($LLMC_SERVER)")
    fs.add("list-models", "bool", False, "Print the local model catalog as JSON and exit")
    fs.add("weights-dir", "string", "",
           "Comma-separated Hugging Face checkpoint dirs (or parents of them) to serve as models ($LLMC_WEIGHTS_DIR)")
    return fs


def register_weights(spec: str) -> List[str]:
    """Register every checkpoint under the comma-separated dirs ``spec`` as a model family."""
    from .models.checkpoint import CheckpointError, register_dir

    names: List[str] = []
    for d in (x for x in (trim_space(p) for p in spec.split(",")) if x):
        try:
            found = register_dir(d)
        except (CheckpointError, OSError, ValueError, KeyError) as e:
            raise CLIError(f"loading checkpoint config from {d}: {e}") from None
        if not found:
            raise CLIError(f"no Hugging Face checkpoint (config.json + *.safetensors) under {d}")
        names.extend(found)
    return names


def _stdin_is_pipe(stdin) -> bool:
    try:
        return not stat.S_ISCHR(os.fstat(stdin.fileno()).st_mode)
    except Exception:  # noqa: BLE001
        return False


def get_prompt(args: List[str], file: str, stdin=None) -> str:
    """main.go:363-393."""
    if args:
        return " ".join(args)
    if file:
        try:
            with open(file, "rb") as f:
                data = f.read()
        except OSError as e:
            raise CLIError(f"reading prompt file: {_go_path_err('open', file, e)}") from None
        return trim_space(data.decode("utf-8", "surrogateescape"))
    stdin = sys.stdin if stdin is None else stdin
    if _stdin_is_pipe(stdin):
        raw = stdin.buffer.read() if hasattr(stdin, "buffer") else stdin.read().encode()
        lines = raw.split(b"\n")
        if lines and lines[-1] == b"":
            lines.pop()
        out = []
        for ln in lines:
            if ln.endswith(b"\r"):  # bufio.ScanLines drops a trailing \r
                ln = ln[:-1]
            if len(ln) > 64 * 1024:
                raise CLIError("reading stdin: bufio.Scanner: token too long")
            out.append(ln.decode("utf-8", "surrogateescape"))
        return "\n".join(out)
    raise CLIError("no prompt provided: use positional argument, --file, or pipe to stdin")


def _go_path_err(op: str, path: str, e: OSError) -> str:
    msg = {2: "no such file or directory", 13: "permission denied", 21: "is a directory"}.get(e.errno, e.strerror or str(e))
    return f"{op} {path}: {msg}"


def parse_flags(argv: List[str], stdout: TextIO = sys.stdout, stderr: TextIO = sys.stderr, stdin=None) -> Config:
    fs = make_flagset()
    v, rest = parse_or_exit(fs, argv, stderr)
    wd = v["weights_dir"] or os.environ.get("LLMC_WEIGHTS_DIR", "")
    if wd:
        register_weights(wd)
    if v["list_models"]:
        stdout.write(dump_catalog())
        raise SystemExit(0)
    if v["version"]:
        stdout.write(f"llm-consensus {get_version()}\n  commit: {commit}\n  built:  {date}\n")
        stdout.flush()
        raise SystemExit(0)
    if v["models"] == "":
        raise CLIError("--models flag is required")
    models = [trim_space(m) for m in v["models"].split(",")]
    cfg = Config(models=models, judge=v["judge"], file=v["file"], output=v["output"], data_dir=v["data_dir"],
                 timeout=float(v["timeout"]), prompt="", quiet=v["quiet"], json=v["json"], no_save=v["no_save"],
                 max_tokens=v["max_tokens"], temperature=v["temperature"], top_p=v["top_p"], top_k=v["top_k"],
                 seed=v["seed"], gpus=v["gpus"], trace=v["trace"], placement=v["placement"],
                 judge_tp=v["judge_tp"], server=v["server"] or os.environ.get("LLMC_SERVER", ""),
                 judge_explicit=any(a.lstrip("-").split("=")[0] == "judge" for a in argv[:len(argv) - len(rest)]))
    cfg.prompt = get_prompt(rest, cfg.file, stdin)
    return cfg


def init_registry(cfg: Config, concurrency: int = 1) -> Registry:
    """main.go:395-438: every model in --models plus the judge must resolve before any query.
    ``concurrency``: consensus requests the local engines are sized for (the server)."""
    needed: List[str] = []
    for m in cfg.models + [cfg.judge]:
        if m not in needed:
            needed.append(m)
    reg = Registry()
    local_specs = []
    for m in needed:
        try:
            spec = resolve(m)
        except UnknownModel as e:
            raise CLIError(f"initializing provider for {m}: {e}") from None
        if spec.provider == PROVIDER_STUB:
            from .provider.stub import StubProvider

            reg.register(m, StubProvider(m))
        elif spec.provider == PROVIDER_LOCAL:
            local_specs.append(spec)
        else:  # hosted API (reference providers)
            from .provider.remote import RemoteError, create

            try:
                reg.register(m, create(m, spec.provider))
            except RemoteError as e:
                raise CLIError(f"initializing provider for {m}: {e}") from None
    if local_specs:
        from .provider.local import LocalBackend

        gpus = [int(x) for x in cfg.gpus.split(",") if x.strip()] if cfg.gpus else None
        counts = {m: cfg.models.count(m) for m in cfg.models}
        try:
            from .parallel.placement import parse_pins

            pins = parse_pins(cfg.placement) if cfg.placement else None
            backend = LocalBackend(local_specs, judge=cfg.judge, gpus=gpus, trace=cfg.trace, counts=counts,
                                   pins=pins, judge_tp=cfg.judge_tp, concurrency=concurrency)
        except Exception as e:  # noqa: BLE001
            raise CLIError(f"initializing provider for {local_specs[0].name}: {e}") from None
        for spec in local_specs:
            reg.register(spec.name, backend.provider(spec.name))
    return reg


def generate_run_id() -> str:
    """main.go:278-285: local time YYYYMMDD-HHMMSS + '-' + 3 random bytes hex."""
    return time.strftime("%Y%m%d-%H%M%S", time.localtime()) + "-" + secrets.token_hex(3)


def run(argv: List[str], stdout: TextIO = sys.stdout, stderr: TextIO = sys.stderr, stdin=None,
        root_ctx: Optional[Context] = None) -> None:
    cfg = parse_flags(argv, stdout, stderr, stdin)
    if cfg.trace:
        from .utils import trace

        trace.enable(True)
        trace.instant("cli_start", cat="startup")
    ctx = root_ctx or Context.background()
    show_ui = ui.is_terminal(stderr) and not cfg.quiet and not cfg.json
    start = time.monotonic()

    if cfg.server:
        out = _run_remote(cfg, ctx, show_ui, stderr)
        _write_outputs(cfg, out, show_ui, start, stdout, stderr, None)
        return
    registry = init_registry(cfg)
    try:
        _run_with_registry(cfg, registry, ctx, show_ui, start, stdout, stderr)
    finally:
        registry.close()


def _request_template(cfg: Config) -> Request:
    return Request(model="", prompt="", max_tokens=cfg.max_tokens or None, temperature=cfg.temperature,
                   top_p=cfg.top_p, top_k=cfg.top_k or None, seed=cfg.seed or None)


def _run_with_registry(cfg: Config, registry: Registry, ctx: Context, show_ui: bool, start: float,
                       stdout: TextIO, stderr: TextIO) -> None:
    if show_ui:
        ui.print_header(stderr, cfg.prompt)
        ui.print_phase(stderr, "Querying models...")
        ui._write(stderr, "\n")

    progress = ui.Progress(stderr, cfg.models, not show_ui)
    progress.start()
    tmpl = _request_template(cfg)
    # Local judge: prefill the template header now and each response block as it completes
    # (SURVEY.md §7.4), so only the last block + trailer remain on the critical path.
    on_resp = None
    try:
        jp = registry.get(cfg.judge)
    except Exception:  # noqa: BLE001
        jp = None
    if jp is not None and hasattr(jp, "open_session") and len(cfg.models) > 1:
        jp.open_session(prompt_header(cfg.prompt))
        on_resp = lambda r: jp.extend_session(response_block(r))  # noqa: E731
    runner = Runner(registry, cfg.timeout, tmpl).with_callbacks(Callbacks(
        on_model_start=progress.model_started,
        on_model_stream=progress.model_streaming,
        on_model_tokens=progress.model_tokens,
        on_model_complete=progress.model_completed,
        on_model_error=progress.model_failed,
        on_model_response=on_resp,
    ))
    try:
        result = runner.run(ctx, cfg.models, cfg.prompt)
    except Exception as e:  # noqa: BLE001
        progress.stop()
        raise CLIError(f"running queries: {e}") from None
    progress.stop()

    if show_ui:
        ui.print_success(stderr, f"Received responses from {len(result.responses)} models")
        ui._write(stderr, "\n")
        ui.print_phase(stderr, "Synthesizing consensus...")
        ui._write(stderr, "\n")

    try:
        judge_provider = registry.get(cfg.judge)
    except Exception as e:  # noqa: BLE001
        raise CLIError(f"judge model {cfg.judge}: {e}") from None
    judge = Judge(judge_provider, cfg.judge, tmpl)
    jprog = ui.Progress(stderr, [cfg.judge], not show_ui)
    jprog.start()
    jprog.model_started(cfg.judge)
    # The judge gets the per-model timeout too (no hidden 60 s cap).
    jctx = ctx.with_timeout(cfg.timeout)
    def judge_stream(chunk: str) -> None:
        jprog.model_streaming(cfg.judge, chunk)

    judge_stream.tokens_hook = lambda n: jprog.model_tokens(cfg.judge, n)  # type: ignore[attr-defined]
    try:
        consensus = judge.synthesize_stream(jctx, cfg.prompt, result.responses, judge_stream)
        err = None
    except Exception as e:  # noqa: BLE001
        consensus, err = "", e
    jprog.model_completed(cfg.judge)
    jprog.stop()
    if err is not None:
        raise CLIError(f"consensus synthesis: {err}")

    if show_ui:
        ui.print_success(stderr, "Consensus reached!")

    out = Result(prompt=cfg.prompt, responses=result.responses, consensus=consensus, judge=cfg.judge,
                 warnings=result.warnings, failed_models=result.failed_models)
    _write_outputs(cfg, out, show_ui, start, stdout, stderr, registry)


def _write_outputs(cfg: Config, out: Result, show_ui: bool, start: float, stdout: TextIO, stderr: TextIO,
                   registry: Optional[Registry]) -> None:
    """Persistence + output routing (main.go:186-273)."""
    consensus = out.consensus
    output_path = ""
    run_dir = ""
    if cfg.output:
        output_path = cfg.output
    elif not cfg.json and not cfg.no_save:
        run_dir = os.path.join(cfg.data_dir, generate_run_id())
        try:
            os.makedirs(run_dir, mode=0o755, exist_ok=True)
        except OSError as e:
            raise CLIError(f"creating run directory: {_go_path_err('mkdir', run_dir, e)}") from None
        output_path = os.path.join(run_dir, "result.json")
        for fname, data, label in (("prompt.txt", cfg.prompt, "prompt"), ("consensus.md", consensus, "consensus")):
            try:
                _write_file(os.path.join(run_dir, fname), data.encode("utf-8", "surrogateescape"))
            except OSError as e:
                if show_ui:
                    ui.print_error(stderr, f"Failed to save {label}: {_go_path_err('open', os.path.join(run_dir, fname), e)}")
        if cfg.trace and registry is not None:
            from .utils import trace

            seen = set()
            for m in registry.models():
                be = getattr(registry.get(m), "backend", None)
                if be is not None and id(be) not in seen:
                    seen.add(id(be))
                    be.collect_traces()
            trace.dump(os.path.join(run_dir, "trace.json"))

    text = encode_result(out)
    if output_path:
        try:
            f = open(output_path, "wb")
        except OSError as e:
            raise CLIError(f"creating output file: {_go_path_err('open', output_path, e)}") from None
        with f:
            f.write(text.encode("utf-8", "surrogateescape"))
        if show_ui:
            ui._write(stderr, "\n")
            ui.print_success(stderr, f"Run saved to {os.path.dirname(output_path) or '.'}")
    elif cfg.json:
        _emit(stdout, text)
    elif show_ui:
        ui._write(stderr, "\n")
        for r in out.responses:
            ui.print_model_response(stderr, r.model, r.provider, r.content, r.latency_s)
        ui.print_consensus(stderr, consensus)
        ui.print_summary(stderr, len(cfg.models), len(out.responses), len(out.failed_models or []),
                         time.monotonic() - start)
        if out.warnings:
            ui._write(stderr, "\n")
            for w in out.warnings:
                ui.print_error(stderr, w)
    else:
        _emit(stdout, text)


def _run_remote(cfg: Config, ctx: Context, show_ui: bool, stderr: TextIO) -> Result:
    """Run the consensus on a warm ``llm-consensus`` server (``server.py``): same phases, UI and
    errors as a local run; the server streams progress as server-sent events."""
    import http.client
    import json
    import urllib.parse

    from .provider.base import Response

    u = urllib.parse.urlsplit(cfg.server if "://" in cfg.server else "http://" + cfg.server)
    body = {"prompt": cfg.prompt, "models": cfg.models, "timeout": cfg.timeout, "stream": True,
            "max_tokens": cfg.max_tokens or None, "temperature": cfg.temperature, "top_p": cfg.top_p,
            "top_k": cfg.top_k or None, "seed": cfg.seed or None}
    if cfg.judge_explicit:
        body["judge"] = cfg.judge
    conn_cls = http.client.HTTPSConnection if u.scheme == "https" else http.client.HTTPConnection
    try:
        conn = conn_cls(u.hostname or "127.0.0.1", u.port, timeout=None)
        conn.request("POST", (u.path.rstrip("/") or "") + "/v1/consensus", body=json.dumps(body).encode(),
                     headers={"Content-Type": "application/json"})
        resp = conn.getresponse()
    except OSError as e:
        raise CLIError(f"connecting to server {cfg.server}: {e}") from None
    if resp.status != 200:
        data = resp.read()
        try:
            msg = json.loads(data)["error"]
        except (ValueError, KeyError, TypeError):
            msg = f"server returned {resp.status}: {data[:200]!r}"
        raise CLIError(msg)

    if show_ui:
        ui.print_header(stderr, cfg.prompt)
        ui.print_phase(stderr, "Querying models...")
        ui._write(stderr, "\n")
    progress = ui.Progress(stderr, cfg.models, not show_ui)
    progress.start()
    jprog = None
    judge_name = cfg.judge
    result_text = None
    error = None
    try:
        name, data = "", []
        while True:
            if ctx.done():
                raise CLIError(f"running queries: {ctx.err()}")
            line = resp.readline()
            if not line:
                break
            line = line.decode("utf-8", "surrogateescape").rstrip("\r\n")
            if line.startswith("event: "):
                name = line[7:]
                continue
            if line.startswith("data: "):
                data.append(line[6:])
                continue
            if line or not name:
                continue
            payload = "\n".join(data)
            ev, name, data = name, "", []
            if ev == "result":
                result_text = payload
                continue
            d = json.loads(payload)
            if ev == "model_start":
                progress.model_started(d["model"])
            elif ev == "chunk":
                progress.model_streaming(d["model"], d["text"])
            elif ev == "tokens":
                progress.model_tokens(d["model"], d["n"])
            elif ev == "model_done":
                progress.model_completed(d["model"])
            elif ev == "model_error":
                progress.model_failed(d["model"], Exception(d["error"]))
            elif ev == "judge_start":
                progress.stop()
                judge_name = d["judge"]
                if show_ui:
                    ui.print_success(stderr, f"Received responses from {d['responses']} models")
                    ui._write(stderr, "\n")
                    ui.print_phase(stderr, "Synthesizing consensus...")
                    ui._write(stderr, "\n")
                jprog = ui.Progress(stderr, [judge_name], not show_ui)
                jprog.start()
                jprog.model_started(judge_name)
            elif ev == "judge_chunk" and jprog is not None:
                jprog.model_streaming(judge_name, d["text"])
            elif ev == "error":
                error = d["error"]
    except (OSError, ValueError, KeyError, http.client.HTTPException) as e:
        error = f"reading server stream: {e}"
    finally:
        progress.stop()
        if jprog is not None:
            jprog.model_completed(judge_name)
            jprog.stop()
        conn.close()
    if error is not None:
        raise CLIError(error)
    if result_text is None:
        raise CLIError(f"server {cfg.server} closed the stream without a result")
    if show_ui:
        ui.print_success(stderr, "Consensus reached!")
    r = json.loads(result_text)
    return Result(prompt=r["prompt"],
                  responses=[Response(model=x["model"], content=x["content"], provider=x["provider"],
                                      latency_ns=int(x["latency_ms"]) * 1_000_000) for x in r["responses"] or []],
                  consensus=r["consensus"], judge=r["judge"], warnings=r.get("warnings"),
                  failed_models=r.get("failed_models"))


def _write_file(path: str, data: bytes) -> None:
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    with os.fdopen(fd, "wb") as f:
        f.write(data)


def _emit(stdout: TextIO, text: str) -> None:
    ui._write(stdout, text)


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    ctx = Context.background()

    def _on_signal(signum, frame):  # main.go:90 signal.NotifyContext(SIGINT, SIGTERM)
        ctx.cancel()

    for s in (signal.SIGINT, signal.SIGTERM):
        try:
            signal.signal(s, _on_signal)
        except ValueError:  # not in main thread
            pass
    try:
        run(argv, root_ctx=ctx)
    except CLIError as e:
        ui._write(sys.stderr, f"error: {e}\n")
        return 1
    except SystemExit as e:
        return int(e.code or 0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
