"""Tensor parallelism through the HIP kernels on ONE GPU: two rank processes share the card
(gloo bootstrap, custom IPC all-reduce / all-gather for the decode collectives, HIP-graph decode)
and must reproduce the TP=1 engine's logits and greedy tokens (SURVEY.md §4.2 TP (b): virtual TP
on one GPU)."""

import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

PROMPT = [(i * 13) % 700 + 256 for i in range(40)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, q, ekw=None):
    import torch.distributed as dist

    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        from llm_consensus_amd.engine import Engine, EngineConfig
        from llm_consensus_amd.models.config import FAMILIES
        from llm_consensus_amd.parallel.comm import TPGroup

        ekw = dict(ekw or {})
        if ekw.pop("_cu_split", False):  # each rank on its own half of the chip (as on GPUs of their own)
            import os

            os.environ["LLMC_CU_MASK"] = f"{rank * 128}-{rank * 128 + 127}"
        tp = TPGroup(dist.group.WORLD, rank, world)
        tp.enable_custom("cuda:0")
        if ekw.pop("_expect_fused", False):
            assert tp.custom_fused is not None
        expect_ao = ekw.pop("_expect_ao", False)
        expect_qa_o = ekw.pop("_expect_qa_o", False)
        e = Engine(FAMILIES[name], EngineConfig(device="cuda:0", max_context=512, seed=5, **ekw), tp=tp)
        if expect_qa_o:  # the one-launch qkv + attention + o_proj runs on this TP rank's buckets
            assert e.qa_o and any(e.qa_plan), (e.qa_o, e.qa_plan)
        if expect_ao:  # the fused attention + o_proj launch runs on this TP rank's decode buckets
            assert all(e.ao_chunks), e.ao_chunks
        e.warmup_graphs()
        s = e.new_sequence()
        e.prefill([s], [PROMPT])
        logits = e.full_logits(s).float().cpu()
        e.free_sequence(s)
        gen = e.generate_ids(PROMPT, 24, temperature=0.0, stop_on_eos=False)
        torch.cuda.synchronize()
        if rank == 0:
            q.put((logits.tolist(), gen, tp.custom_timed_out()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put((repr(ex) + traceback.format_exc(), None, True))


@pytest.mark.parametrize("name,ekw", [
    ("llama-small", {}), ("mixtral-tiny", {}),
    ("llama-small", {"sp_min_tokens": 16}),                            # sequence-parallel prefill
    ("mixtral-tiny", {"expert_parallel": True}),                       # EP: localized ids in the graphs
    ("mixtral-tiny", {"expert_parallel": True, "sp_min_tokens": 16}),  # EP + SP: all-to-all dispatch
])
def test_tp2_gpu_matches_tp1(cuda, name, ekw):
    _tp2_vs_tp1(name, ekw)


def test_tp2_gpu_fused_rowparallel_allreduce_matches_tp1(cuda, monkeypatch):
    """The TP engine's decode with the all-reduce fused into the row-parallel GEMVs (EPI_AR, forced
    on although the two ranks share the GPU: llama-small's grids all fit on the chip at once)."""
    monkeypatch.setenv("LLMC_FUSED_AR", "force")
    _tp2_vs_tp1("llama-small", {"_expect_fused": True})


def test_tp2_gpu_fused_allreduce_cu_partitioned_matches_tp1(cuda, monkeypatch):
    """The fused row-parallel all-reduce with each rank's engine streams on its own half of the
    chip (EngineConfig.cu_mask via LLMC_CU_MASK, as scripts/tp_rehearsal.py runs a TP group)."""
    monkeypatch.setenv("LLMC_FUSED_AR", "force")
    _tp2_vs_tp1("llama-small", {"_expect_fused": True, "_cu_split": True})


def test_tp2_gpu_attn_oproj_fused_allreduce_matches_tp1(cuda, monkeypatch):
    """TP ranks on the one-launch attention + o_proj (every bucket: LLMC_ATTN_OPROJ=all) with the
    all-reduce in the kernel's tile-reducer epilogue (attn_oproj.hip, car_proto.h push protocol),
    each rank on its own half of the chip."""
    monkeypatch.setenv("LLMC_FUSED_AR", "force")
    monkeypatch.setenv("LLMC_ATTN_OPROJ", "all")
    monkeypatch.setenv("LLMC_TP_ATTN_OPROJ", "1")
    _tp2_vs_tp1("llama-small", {"_expect_fused": True, "_cu_split": True, "_expect_ao": True})


def test_tp2_gpu_attn_oproj_separate_allreduce_matches_tp1(cuda, monkeypatch):
    """... and with the rank's partial (rank 0: + residual) followed by the group's all-reduce launch."""
    monkeypatch.setenv("LLMC_FUSED_AR", "0")
    monkeypatch.setenv("LLMC_ATTN_OPROJ", "all")
    monkeypatch.setenv("LLMC_TP_ATTN_OPROJ", "1")
    _tp2_vs_tp1("llama-small", {"_expect_ao": True})


def test_tp2_gpu_qkv_attn_o_fused_allreduce_matches_tp1(cuda, monkeypatch):
    """TP ranks on the one-launch qkv + attention + o_proj (the o-role of qkv_attn.hip) with the
    all-reduce in the o-role's epilogue, each rank on its own half of the chip."""
    monkeypatch.setenv("LLMC_FUSED_AR", "force")
    monkeypatch.setenv("LLMC_QKV_ATTN_O", "1")
    _tp2_vs_tp1("llama-small", {"_expect_fused": True, "_cu_split": True, "_expect_qa_o": True})


def test_tp2_gpu_qkv_attn_o_separate_allreduce_matches_tp1(cuda, monkeypatch):
    """... and with the rank's o_proj share (rank 0: + residual) followed by the all-reduce launch."""
    monkeypatch.setenv("LLMC_FUSED_AR", "0")
    monkeypatch.setenv("LLMC_QKV_ATTN_O", "1")
    _tp2_vs_tp1("llama-small", {"_expect_qa_o": True})


def _tp2_vs_tp1(name, ekw):
    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.models.config import FAMILIES

    ref = Engine(FAMILIES[name], EngineConfig(device="cuda:0", max_context=512, seed=5))
    s = ref.new_sequence()
    ref.prefill([s], [PROMPT])
    ref_logits = ref.full_logits(s).float().cpu()
    ref.free_sequence(s)
    ref_gen = ref.generate_ids(PROMPT, 24, temperature=0.0, stop_on_eos=False)
    del ref
    torch.cuda.empty_cache()

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, name, q, ekw)) for r in range(2)]
    for p in procs:
        p.start()
    logits, gen, tmo = q.get(timeout=400)
    for p in procs:
        p.join(timeout=120)
    assert not isinstance(logits, str), logits
    assert not tmo
    logits = torch.tensor(logits)
    d = (logits - ref_logits).abs()
    bad = (d > 0.05 * ref_logits.abs().max()).nonzero().flatten()
    assert bad.numel() == 0, (f"{bad.numel()} of {d.numel()} logits off (max {d.max().item():.3f}); first "
                              f"{bad[:8].tolist()} last {bad[-8:].tolist()}; got {logits[bad[:8]].tolist()} "
                              f"want {ref_logits[bad[:8]].tolist()}")
    # greedy continuation: equal until the first numerical near-tie, which the TP=1 model must
    # confirm (teacher-forced: its logits at the diverging position put the TP token within noise
    # of its own argmax)
    agree = 0
    for a, b in zip(gen, ref_gen):
        if a != b:
            break
        agree += 1
    if agree < 8:
        ref = Engine(FAMILIES[name], EngineConfig(device="cuda:0", max_context=512, seed=5))
        s = ref.new_sequence()
        ref.prefill([s], [PROMPT + gen[:agree]])
        lt = ref.full_logits(s).float().cpu()
        gap = float(lt.max() - lt[gen[agree]])
        assert gap < 0.01 * float(lt.abs().max()), (agree, gap, gen, ref_gen)


def _rccl_capture_worker(port, q):
    import torch.distributed as dist

    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        from llm_consensus_amd.parallel.comm import TPGroup, rccl_graph_capture, rccl_graph_replay_check

        cap = rccl_graph_capture(dist.group.WORLD, 0, 1, "cuda:0")
        ok = cap is not None and rccl_graph_replay_check(cap, 0, 1, "cuda:0")
        # the collective wrapper on a gloo group is never capturable
        g = dist.new_group([0], backend="gloo")
        gloo_ok = TPGroup(g, 0, 2).graph_capture_ok("cuda:0")
        dist.destroy_process_group()
        q.put((ok, gloo_ok))
    except Exception as e:  # noqa: BLE001
        q.put((f"{type(e).__name__}: {e}", None))


def test_rccl_collectives_capture_in_hip_graph():
    """The RCCL fallback of TP decode (peers not mappable) captures its collectives in the decode
    graph after a self-check: an all-reduce + all-gather captured in a HIP graph and replayed give
    the right sums on this torch/RCCL build (one rank: more need more GPUs than the test box has)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_capture_worker, args=(_free_port(), q))
    p.start()
    ok, gloo_ok = q.get(timeout=300)
    p.join(timeout=60)
    assert ok is True, ok
    assert gloo_ok is False
