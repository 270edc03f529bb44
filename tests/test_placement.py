"""Placement solver on the BASELINE.json configs (SURVEY.md §4.2 "Scheduler: placement solver
unit tests"; rules in llm_consensus_amd/parallel/placement.py). Pure CPU: demands are sized from
the public architecture shapes, 288 GB of HBM per GPU."""

import pytest

from llm_consensus_amd.parallel.placement import ModelDemand, PlacementError, describe, solve

G = 10**9
W8B, W70B, WMIX, WPHI = 16 * G, 141 * G, 93 * G, 8 * G  # bf16 weights (GiB -> GB)


def test_config2_three_8b_responders_plus_judge_on_four_gpus():
    ds = [ModelDemand(f"llama-3-8b@{i}", W8B, 2 * G) for i in range(3)]
    ds.append(ModelDemand("llama-3-8b@judge", W8B, 8 * G, is_judge=True))
    p = solve(ds, list(range(4)))
    # one engine per GPU: the responders spread out, the judge takes the free GPU
    assert sorted(g[0] for g in p.gpus.values()) == [0, 1, 2, 3]
    assert p.gpus["llama-3-8b@judge"] == [3]


def test_config3_eight_responders_judge_time_shares_gpu0():
    ds = [ModelDemand(f"llama-3-8b@{i}", W8B, 2 * G) for i in range(8)]
    ds.append(ModelDemand("llama-3-8b@judge", W8B, 10 * G, is_judge=True))
    p = solve(ds, list(range(8)))
    assert sorted(p.gpus[f"llama-3-8b@{i}"][0] for i in range(8)) == list(range(8))
    assert p.gpus["llama-3-8b@judge"] == [0]  # no free GPU: lowest id, own hipStream
    assert p.models_on(0) == ["llama-3-8b@0", "llama-3-8b@judge"]


def test_config4_two_70b_tp4_on_disjoint_halves():
    ds = [ModelDemand("llama-3-70b@0", W70B, 20 * G, tp=4), ModelDemand("llama-3-70b@1", W70B, 20 * G, tp=4),
          ModelDemand("llama-3-8b@judge", W8B, 5 * G, is_judge=True)]
    p = solve(ds, list(range(8)))
    groups = sorted(p.gpus["llama-3-70b@0"] + p.gpus["llama-3-70b@1"])
    assert groups == list(range(8))
    assert {tuple(p.gpus["llama-3-70b@0"]), tuple(p.gpus["llama-3-70b@1"])} == {(0, 1, 2, 3), (4, 5, 6, 7)}
    assert p.gpus["llama-3-8b@judge"] == [0]  # every GPU busy: spare stream on the lowest
    assert "llama-3-70b@0->" in describe(p)


def test_config5_mixed_fleet_with_70b_tp4_judge():
    ds = [ModelDemand("mixtral-8x7b", WMIX, 5 * G), ModelDemand("llama-3-8b", W8B, 2 * G),
          ModelDemand("phi-3-mini", WPHI, 6 * G), ModelDemand("llama-3-70b@judge", W70B, 30 * G, tp=4, is_judge=True)]
    p = solve(ds, list(range(8)))
    assert p.gpus["llama-3-70b@judge"] == [0, 1, 2, 3]  # TP groups first, aligned
    singles = [p.gpus[m][0] for m in ("mixtral-8x7b", "llama-3-8b", "phi-3-mini")]
    assert len(set(singles)) == 3 and all(g >= 4 for g in singles)  # the free half, one each


def test_memory_is_checked_per_gpu():
    # 70B unsharded (141 GB) + 130 GB of KV = 271 GB does not fit one 288 GB GPU's usable 92 % (265 GB)
    with pytest.raises(PlacementError, match="no GPU has that free"):
        solve([ModelDemand("llama-3-70b", W70B, 130 * G)], [0])
    # fits once it is TP=2 (135.5 GB per GPU)
    p = solve([ModelDemand("llama-3-70b", W70B, 130 * G, tp=2)], [0, 1])
    assert p.gpus["llama-3-70b"] == [0, 1]
    # co-location fills the least-loaded GPU until memory runs out
    ds = [ModelDemand(f"m{i}", 100 * G, 0) for i in range(5)]
    with pytest.raises(PlacementError):
        solve(ds, [0, 1])


def test_tp_larger_than_node_and_no_gpus():
    with pytest.raises(PlacementError, match="tp=8"):
        solve([ModelDemand("llama-3-70b", W70B, 0, tp=8)], list(range(4)))
    with pytest.raises(PlacementError, match="no GPUs"):
        solve([ModelDemand("x", 1, 0)], [])


def test_kv_pool_blocks_fit_the_gpu():
    """16 requests in flight on one GPU: 2 x 8B responders (16 rows each) + an 8B judge (17
    sessions at a 131k context would ask for ~290 GB of KV): every pool shrinks to the GPU's HBM
    left after the weights, pro rata, never below one full context; small asks stay whole."""
    from llm_consensus_amd.catalog import resolve as resolve_model
    from llm_consensus_amd.parallel.placement import HBM_BYTES, USABLE_FRACTION, Placement
    from llm_consensus_amd.provider.local import JUDGE_CONTEXT, KV_BLOCK, RESPONDER_CONTEXT, kv_pool_blocks

    names = ["llama-3-8b@0", "llama-3-8b@1", "llama-3-8b@judge"]
    specs = {n: resolve_model(n) for n in names}
    ctx = {"llama-3-8b@0": RESPONDER_CONTEXT, "llama-3-8b@1": RESPONDER_CONTEXT, "llama-3-8b@judge": JUDGE_CONTEXT}
    pl = Placement({n: [0] for n in names})
    seqs = {"llama-3-8b@0": 16, "llama-3-8b@1": 16, "llama-3-8b@judge": 17}
    blocks = kv_pool_blocks(pl, specs, ctx, seqs)
    per_tok = specs["llama-3-8b@0"].config.kv_bytes_per_token()
    weights = sum(specs[n].config.weight_bytes() for n in names)
    kv = sum(b * KV_BLOCK * per_tok for b in blocks.values())
    assert weights + kv <= HBM_BYTES * USABLE_FRACTION * 1.01
    for n in names:
        assert blocks[n] * KV_BLOCK >= ctx[n]  # at least one full context
    assert blocks["llama-3-8b@judge"] < seqs["llama-3-8b@judge"] * JUDGE_CONTEXT // KV_BLOCK
    # one request in flight: the asks fit, every engine gets all it asked for
    one = kv_pool_blocks(pl, specs, ctx, {"llama-3-8b@0": 1, "llama-3-8b@1": 1, "llama-3-8b@judge": 2})
    assert one["llama-3-8b@judge"] * KV_BLOCK >= 2 * JUDGE_CONTEXT


def test_decode_row_caps_match_the_kernels():
    """The driver's per-engine decode-row cap (torch-free) equals the op layer's limits."""
    from llm_consensus_amd import ops
    from llm_consensus_amd.models.config import FAMILIES
    from llm_consensus_amd.provider import local

    assert local.DECODE_ROWS_MAX == ops.GEMV_MAX_M
    assert local.MOE_DECODE_ROWS_MAX == ops.MOE_GEMVM_MAX_TOKENS
    assert local.max_decode_rows(FAMILIES["mixtral-8x7b"]) == 16
    assert local.max_decode_rows(FAMILIES["llama-3-8b"]) == 32


def test_driver_process_stays_torch_free():
    """The CLI / server driver plans placement and spawns the GPU workers without importing torch
    (its ~2 s import would sit on the startup path before any worker starts)."""
    import subprocess
    import sys

    code = ("import sys, llm_consensus_amd.cli, llm_consensus_amd.provider.local, "
            "llm_consensus_amd.runtime.worker, llm_consensus_amd.server, llm_consensus_amd.parallel.placement; "
            "print('torch' in sys.modules)")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "False"


@pytest.mark.gpu
def test_visible_gpu_count_matches_the_hip_runtime():
    """The driver's torch-free GPU count (KFD topology + accessible render nodes + visibility
    env) equals what the HIP runtime enumerates."""
    import torch

    from llm_consensus_amd.parallel.placement import visible_gpu_count

    assert visible_gpu_count() == torch.cuda.device_count()


def test_visible_gpu_count_from_kfd_topology(tmp_path, monkeypatch):
    """CPU nodes (gpu_id 0) and GPUs whose render node this process cannot open are not counted;
    a visibility variable narrows the count; no topology -> -1 (torch decides)."""
    import os

    from llm_consensus_amd.parallel import placement

    for i, (gid, minor) in enumerate([(0, None), (4242, 128), (5151, 129), (6363, 130)]):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "gpu_id").write_text(f"{gid}\n")
        (d / "properties").write_text("cpu_cores_count 0\n" + (f"drm_render_minor {minor}\n" if minor else ""))
    monkeypatch.setattr(placement, "_KFD_NODES", str(tmp_path))
    real_open = os.open

    def fake_open(p, flags, *a):  # renderD130 is denied (e.g. by the device cgroup): open fails
        if p in ("/dev/dri/renderD128", "/dev/dri/renderD129"):
            return real_open(os.devnull, os.O_RDONLY)
        if p.startswith("/dev/dri/"):
            raise PermissionError(p)
        return real_open(p, flags, *a)

    monkeypatch.setattr(placement.os, "open", fake_open)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert placement.visible_gpu_count() == 2
    assert placement.default_gpus() == [0, 1]
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert placement.visible_gpu_count() == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "-1")  # hides every GPU
    assert placement.visible_gpu_count() == 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1,7,0")  # the runtime stops at the invalid index 7
    assert placement.visible_gpu_count() == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "GPU-1234abcd")  # a UUID: the runtime resolves it
    assert placement.visible_gpu_count() == -1
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.setattr(placement, "_KFD_NODES", str(tmp_path / "missing"))
    assert placement.visible_gpu_count() == -1


def test_fused_allreduce_rule_follows_the_placement():
    """the product workers take the fused row-parallel all-reduce from the placement, by
    the same rule as bench.colocated_tp — a TP engine placed beside an engine that decodes at the
    same time keeps separate all-reduce launches; a judge alone in its phase keeps the fused one."""
    import importlib.util
    import os

    from llm_consensus_amd.parallel.placement import ModelDemand, fused_ar_allowed, fused_ar_plan, solve

    G = 10**9
    # a TP=2 responder and a single-GPU responder on 2 GPUs: the solver puts them together
    p = solve([ModelDemand("big", 40 * G, G, tp=2), ModelDemand("small", 16 * G, G, tp=1),
               ModelDemand("judge", 16 * G, G, tp=2, is_judge=True)], [0, 1])
    assert set(p.gpus["small"]) & set(p.gpus["big"])
    plan = fused_ar_plan(p.gpus, "judge", concurrency=1)
    assert plan["big"] is False          # decodes beside "small"
    assert plan["small"] is True         # single GPU: no all-reduce at all
    assert plan["judge"] is True         # decodes after the responders, alone
    assert fused_ar_plan(p.gpus, "judge", concurrency=2)["judge"] is False  # server: overlaps responders
    # a TP group with its GPUs to itself keeps the fused form
    q = {"a": [0, 1], "b": [2], "c": [3]}
    assert fused_ar_plan(q, None)["a"] is True and fused_ar_allowed(q, "a", ["b", "c"]) is True
    # bench.py uses the same rule for its responder plan (N=2: the third responder is TP=2)
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    plan2 = [{"ranks": [0]}, {"ranks": [1]}, {"ranks": [0, 1]}]
    assert bench.colocated_tp(plan2, [2]) is True and bench.colocated_tp(plan2, [0]) is False
    assert bench.colocated_tp([{"ranks": [0, 1]}, {"ranks": [2]}], [0]) is False


def test_lone_engine_rule_follows_the_placement():
    """Engines that decode with no other engine on their GPUs take the lone-engine launch forms
    (the fused attention + o_proj in every context bucket, ops.attn_oproj_min_chunk); co-located
    responders keep the default. bench.py's responder_alone applies the same rule."""
    import importlib.util
    import os

    from llm_consensus_amd import ops
    from llm_consensus_amd.parallel.placement import alone_plan, decodes_alone

    one_gpu = {"r0": [0], "r1": [0], "r2": [0], "judge": [0]}  # BASELINE config 2 on one GPU
    plan = alone_plan(one_gpu, "judge")
    assert plan == {"r0": False, "r1": False, "r2": False, "judge": True}
    assert alone_plan(one_gpu, "judge", concurrency=2)["judge"] is False  # server: overlaps
    eight = {f"r{i}": [i] for i in range(8)}
    eight["judge"] = list(range(8))  # config 3 at N=8: one responder per GPU, TP=8 judge
    plan8 = alone_plan(eight, "judge")
    assert all(plan8[f"r{i}"] for i in range(8)) and plan8["judge"]
    assert decodes_alone({"a": [0, 1], "b": [1]}, "a", ["b"]) is False
    assert ops.attn_oproj_min_chunk(True) == 32
    if os.environ.get("LLMC_ATTN_OPROJ") != "all":
        assert ops.attn_oproj_min_chunk(False) == ops.ATTN_OPROJ_MIN_CHUNK
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.responder_alone([{"ranks": [0]}, {"ranks": [0]}, {"ranks": [0]}], [0]) is False
    assert bench.responder_alone([{"ranks": [0]}, {"ranks": [1]}, {"ranks": [2]}], [1]) is True
    # the one-GPU rehearsal puts every rank on cuda:0: nobody is alone there
    os.environ["LLMC_BENCH_SAME_GPU"] = "1"
    try:
        assert bench.responder_alone([{"ranks": [0]}, {"ranks": [1]}, {"ranks": [2]}], [1]) is False
    finally:
        del os.environ["LLMC_BENCH_SAME_GPU"]


def test_judge_that_also_responds_is_treated_as_a_responder():
    """a judge named in --models decodes during the fan-out too. Pinned (--judge-tp)
    onto the responders' GPUs it must neither take the fused row-parallel all-reduce nor the
    lone-engine launch forms, and the responders beside it are not alone either."""
    from llm_consensus_amd.parallel.placement import alone_plan, fused_ar_plan

    gpus = {"judge": [0, 1], "r1": [1], "r2": [2]}
    # judge-only: it decodes after the fan-out, alone on its GPUs
    assert fused_ar_plan(gpus, "judge")["judge"] is True
    assert alone_plan(gpus, "judge")["judge"] is True
    assert alone_plan(gpus, "judge")["r1"] is True  # the judge does not decode during the fan-out
    # the judge also answers: it shares GPU 1 with r1 while both decode
    resp = ["judge", "r1", "r2"]
    assert fused_ar_plan(gpus, "judge", responders=resp)["judge"] is False
    a = alone_plan(gpus, "judge", responders=resp)
    assert a["judge"] is False and a["r1"] is False and a["r2"] is True
    # a judge that answers but shares no GPU stays alone
    assert alone_plan({"judge": [0], "r1": [1]}, "judge", responders=["judge", "r1"])["judge"] is True
