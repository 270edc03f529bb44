"""Placement solver: which GPU(s) host each model engine (T3).

Replaces "the remote API's job". Inputs: the distinct local models of a run (responders + judge),
each with a TP degree, and the node's GPUs (288 GB HBM3E each). Rules:
  1. TP groups first, on contiguous, aligned GPU ranges (xGMI is fully connected, but aligned
     groups {0-3},{4-7} keep two TP=4 models on disjoint halves — BASELINE config 4);
  2. single-GPU responders spread over the GPUs with the fewest engines (one replica per GPU
     when possible: decode is HBM-bound, co-located engines share bandwidth);
  3. the judge goes to the least-loaded GPU (a free GPU if any; else GPU 0, time-sharing via its
     own hipStream — BASELINE config 3);
  4. memory check: weights + KV pool must fit in the usable HBM of every GPU it touches.
"""

from __future__ import annotations

import dataclasses
import os
from typing import Dict, List, Optional, Sequence

HBM_BYTES = 288 * 10**9
USABLE_FRACTION = 0.92


@dataclasses.dataclass
class ModelDemand:
    name: str
    weight_bytes: int
    kv_bytes: int
    tp: int = 1
    is_judge: bool = False


@dataclasses.dataclass
class Placement:
    gpus: Dict[str, List[int]]  # model name -> GPU ids (len == tp)

    def models_on(self, gpu: int) -> List[str]:
        return [m for m, g in self.gpus.items() if gpu in g]

    def used_gpus(self) -> List[int]:
        return sorted({g for gs in self.gpus.values() for g in gs})


class PlacementError(Exception):
    pass


def decodes_alone(gpus: Dict[str, List[int]], name: str, concurrent: Sequence[str]) -> bool:
    """Does engine ``name`` decode with none of its GPUs shared by an engine that decodes at the
    same time (``concurrent``)? Such an engine's latency-bound kernels have the chip to
    themselves (no other stream fills their ramps), which changes which launch forms pay."""
    mine = set(gpus[name])
    return not any(mine & set(gpus[o]) for o in concurrent if o != name and o in gpus)


def fused_ar_allowed(gpus: Dict[str, List[int]], name: str, concurrent: Sequence[str]) -> bool:
    """May tensor-parallel engine ``name`` run its row-parallel decode all-reduce inside the GEMV
    epilogue (``EngineConfig.fused_ar``)? Not when an engine that decodes at the same time
    (``concurrent``) shares one of its GPUs: the fused launch's ~256 blocks per GPU spin on the peer
    GPUs while holding CUs, and a co-located engine's blocks queued behind them delay the very
    peers they wait for. Single-GPU engines have no all-reduce (True)."""
    if len(gpus[name]) <= 1:
        return True
    return decodes_alone(gpus, name, concurrent)


def _concurrent(gpus: Dict[str, List[int]], m: str, judge: Optional[str], concurrency: int,
                responders: Optional[Sequence[str]] = None) -> List[str]:
    """The engines that decode while ``m`` does in a consensus run: the responders decode
    together; the judge decodes after the last response (runner.go:118 then judge.go:96), so with
    one request in flight it overlaps nothing — with several (the server) one request's judge
    overlaps the next one's responders. ``responders`` = the engines that answer the fan-out
    (default: every engine but the judge). A judge that is also a responder (``--models`` names
    it: LocalBackend gives it rows of its own) decodes during the fan-out too, so it is treated as
    any other responder: its engine's launch forms are fixed for both phases."""
    if concurrency > 1:
        return [o for o in gpus if o != m]
    resp = set(responders) if responders is not None else {o for o in gpus if o != judge}
    if m not in resp:
        return []
    return [o for o in gpus if o != m and o in resp]


def fused_ar_plan(gpus: Dict[str, List[int]], judge: Optional[str], concurrency: int = 1,
                  responders: Optional[Sequence[str]] = None) -> Dict[str, bool]:
    """``fused_ar_allowed`` for every placed engine of a consensus run (``_concurrent``)."""
    return {m: fused_ar_allowed(gpus, m, _concurrent(gpus, m, judge, concurrency, responders)) for m in gpus}


def alone_plan(gpus: Dict[str, List[int]], judge: Optional[str], concurrency: int = 1,
               responders: Optional[Sequence[str]] = None) -> Dict[str, bool]:
    """``decodes_alone`` for every placed engine of a consensus run (``_concurrent``): the engines
    that take the lone-engine launch forms (``EngineConfig.attn_oproj_min_chunk``)."""
    return {m: decodes_alone(gpus, m, _concurrent(gpus, m, judge, concurrency, responders)) for m in gpus}


def parse_pins(spec: str) -> Dict[str, List[int]]:
    """``--placement`` syntax: ``model=g[+g...][,model=g...]`` (a '+'-joined list is a TP group)."""
    pins: Dict[str, List[int]] = {}
    for item in filter(None, (x.strip() for x in (spec or "").split(","))):
        name, sep, gs = item.rpartition("=")
        if not sep or not name.strip():
            raise PlacementError(f"bad placement entry {item!r} (want model=gpu[+gpu...])")
        try:
            ids = [int(x) for x in gs.split("+")]
        except ValueError:
            raise PlacementError(f"bad GPU list in placement entry {item!r}") from None
        if len(set(ids)) != len(ids):
            raise PlacementError(f"duplicate GPU in placement entry {item!r}")
        pins[name.strip()] = ids
    return pins


def solve(demands: Sequence[ModelDemand], gpu_ids: Sequence[int], hbm_bytes: int = HBM_BYTES,
          pins: Optional[Dict[str, List[int]]] = None) -> Placement:
    """Place every demand; ``pins`` (``--placement``) fixes some models' GPUs first — a pinned
    list of n GPUs makes that model TP=n — and the rules below place the rest around them."""
    gpu_ids = list(gpu_ids)
    if not gpu_ids:
        raise PlacementError("no GPUs available")
    cap = hbm_bytes * USABLE_FRACTION
    used = {g: 0.0 for g in gpu_ids}
    count = {g: 0 for g in gpu_ids}
    out: Dict[str, List[int]] = {}
    pins = dict(pins or {})
    unknown = sorted(set(pins) - {d.name for d in demands})
    if unknown:
        raise PlacementError(f"placement names models not in the run: {unknown}")

    def fits(g: int, b: float) -> bool:
        return used[g] + b <= cap

    def take(name: str, gs: List[int], per_gpu: float) -> None:
        for g in gs:
            used[g] += per_gpu
            count[g] += 1
        out[name] = gs

    # 0. pinned models, as given
    for d in demands:
        gs = pins.get(d.name)
        if gs is None:
            continue
        bad = [g for g in gs if g not in used]
        if bad:
            raise PlacementError(f"{d.name}: placement GPU(s) {bad} not available (have {gpu_ids})")
        per = (d.weight_bytes + d.kv_bytes) / len(gs)
        if not all(fits(g, per) for g in gs):
            raise PlacementError(f"{d.name}: {per / 1e9:.1f} GB per GPU does not fit on {gs}")
        take(d.name, list(gs), per)
    demands = [dataclasses.replace(d) for d in demands if d.name not in pins]
    # 1. tensor-parallel models: aligned contiguous groups, least-loaded group first
    for d in sorted((d for d in demands if d.tp > 1), key=lambda d: -d.tp):
        if d.tp > len(gpu_ids):
            raise PlacementError(f"{d.name}: tp={d.tp} needs {d.tp} GPUs, only {len(gpu_ids)} available")
        per = (d.weight_bytes + d.kv_bytes) / d.tp
        groups = [gpu_ids[i:i + d.tp] for i in range(0, len(gpu_ids) - d.tp + 1, d.tp)]
        groups = [g for g in groups if all(fits(x, per) for x in g)]
        if not groups:
            raise PlacementError(f"{d.name}: no GPU group with {per / 1e9:.1f} GB free per GPU")
        best = min(groups, key=lambda g: (sum(count[x] for x in g), g[0]))
        take(d.name, best, per)
    # 2. single-GPU responders, then 3. the judge
    singles = [d for d in demands if d.tp == 1 and not d.is_judge] + [d for d in demands if d.tp == 1 and d.is_judge]
    for d in singles:
        per = d.weight_bytes + d.kv_bytes
        cands = [g for g in gpu_ids if fits(g, per)]
        if not cands:
            raise PlacementError(f"{d.name}: needs {per / 1e9:.1f} GB, no GPU has that free")
        best = min(cands, key=lambda g: (count[g], used[g], g))
        take(d.name, [best], per)
    return Placement(out)


def describe(p: Placement) -> str:
    return "; ".join(f"{m}->{','.join(map(str, g))}" for m, g in sorted(p.gpus.items()))


_KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def visible_gpu_count() -> int:
    """GPUs this process can open, without importing torch (the driver process stays torch-free;
    the import alone is ~1.5 s on the CLI's startup path): KFD topology nodes with a GPU whose
    render node is accessible, narrowed by HIP/ROCR/CUDA_VISIBLE_DEVICES as the HIP runtime
    narrows them. -1 when the topology is unreadable (the caller asks torch instead)."""
    try:
        nodes = sorted(os.listdir(_KFD_NODES), key=lambda d: int(d) if d.isdigit() else 1 << 30)
    except OSError:
        return -1
    n = 0
    for d in nodes:
        try:
            with open(os.path.join(_KFD_NODES, d, "gpu_id")) as f:
                if int(f.read().strip() or "0") == 0:
                    continue  # a CPU node
            minor = None
            with open(os.path.join(_KFD_NODES, d, "properties")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "drm_render_minor":
                        minor = int(v)
            if minor is None:
                continue
            # open, not os.access: a device-cgroup denial only shows when the node is opened
            fd = os.open(f"/dev/dri/renderD{minor}", os.O_RDWR | os.O_CLOEXEC)
            os.close(fd)
            n += 1
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None:
            continue
        # the runtime keeps the leading valid device indices and stops at the first invalid one
        # ("-1" hides every GPU); non-index forms (UUIDs) are the runtime's to resolve: ask it
        kept = 0
        for x in (t.strip() for t in v.split(",")):
            if x == "":
                continue
            if not x.lstrip("-").isdigit():
                return -1
            if not 0 <= int(x) < n:
                break
            kept += 1
        n = min(n, kept)
    return n


def default_gpus(requested: Optional[List[int]] = None) -> List[int]:
    if requested:
        return list(requested)
    n = visible_gpu_count()
    if n <= 0:  # unreadable topology, or no render node passed the access check: ask the runtime
        try:
            import torch

            n = torch.cuda.device_count()  # does not initialise the GPU on this image
        except Exception:  # noqa: BLE001
            n = 0
    return list(range(n))
