"""A tensor-parallel rank that stops mid-decode ("a dead TP rank fails that
engine, not the run"; reference per-model failure ``internal/runner/runner.go:100-107``).

Rank 1 of a TP=2 engine raises before one of its decode replays, so it never launches the
collectives its peer's replay waits on. The survivor's fused row-parallel all-reduce spins must give
up within their 1-s bound (csrc/kernels/car_proto.h ``car_spin``), the group must agree on the
failure at the same replay (``TPGroup.step_agree``), both requests must fail within 10 s, and after
the collective resync a new request must reproduce a clean run's tokens bit for bit.

Two layouts: both ranks on ONE GPU, each on its own half of the CUs (``LLMC_CU_MASK``, fused
all-reduce forced: ``LLMC_FUSED_AR=force``), as the rehearsals run a TP group; and — gated on
``torch.cuda.device_count() >= 2`` — rank i on ``cuda:i`` over RCCL.

Two more cases, on the one-GPU layout: a rank that STALLS for longer than the spin bound
and then goes on (both requests fail at the replay where the survivor's spin gave up, and no token
computed after the give-up is streamed on either rank), and a prefill that runs longer than the
host's replay deadline (``Engine.stall_s``): the decode waits for it instead of aborting the group."""

import os
import socket
import time

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


def _worker(rank, world, port, layout, q, case="dead"):
    import datetime

    import torch.distributed as dist

    try:
        os.environ["LLMC_FUSED_AR"] = "force" if layout == "cu_split" else "1"
        if layout == "cu_split":
            os.environ["LLMC_CU_MASK"] = f"{rank * 128}-{rank * 128 + 127}"
            dev = "cuda:0"
            torch.cuda.set_device(0)
            dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=60))
            ctrl = dist.group.WORLD
        else:
            dev = f"cuda:{rank}"
            torch.cuda.set_device(rank)
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", rank))
            ctrl = dist.new_group(list(range(world)), backend="gloo", timeout=datetime.timedelta(seconds=60))
        from llm_consensus_amd.engine import Engine, EngineConfig, EngineError
        from llm_consensus_amd.models.config import FAMILIES
        from llm_consensus_amd.parallel.comm import TPGroup

        tp = TPGroup(dist.group.WORLD, rank, world, ctrl=ctrl)
        assert tp.enable_custom(dev) and tp.custom_fused is not None
        e = Engine(FAMILIES["llama-small"], EngineConfig(device=dev, max_context=1024, seed=5), tp=tp)
        e.warmup_graphs()
        ref = e.generate_ids(PROMPT, 24, temperature=0.0, stop_on_eos=False)
        if case == "long_prefill":
            q.put((rank,) + _long_prefill(e, ref))
            dist.barrier()
            dist.destroy_process_group()
            return
        if case == "stall":
            q.put((rank,) + _stall(e, tp, rank))
            dist.barrier()
            dist.destroy_process_group()
            return
        checks = []
        orig = tp.check_collectives

        def check():
            ok = orig()
            checks.append(ok)
            return ok

        tp.check_collectives = check
        if rank == 1:
            e.fault_at = ("decode", 100)  # stops before the replay that would produce token 100
        t0 = time.monotonic()
        err = None
        try:
            e.generate_ids(PROMPT, 600, temperature=0.0, stop_on_eos=False)
        except EngineError as ex:
            err = f"{type(ex).__name__}: {ex}"
        dt = time.monotonic() - t0
        again = e.generate_ids(PROMPT, 24, temperature=0.0, stop_on_eos=False)
        torch.cuda.synchronize()
        q.put((rank, err, dt, again == ref, checks, tp.custom_timed_out()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put((rank, repr(ex) + traceback.format_exc(), -1.0, False, [], True))


def _stall(e, tp, rank):
    """Rank 1 sleeps 3 s (> the 1-s spin bound) before the replay that would produce token 100,
    then goes on. -> (error, seconds, streamed tokens, clean-run tokens, request after resync ok)."""
    from llm_consensus_amd.engine import EngineError

    long_ref = e.generate_ids(PROMPT, 200, temperature=0.0, stop_on_eos=False)
    if rank == 1:
        e.fault_at = ("decode", 100, 3.0)
    streamed = []
    t0 = time.monotonic()
    err = None
    try:
        e.generate_ids(PROMPT, 600, temperature=0.0, stop_on_eos=False, on_tokens=streamed.extend)
    except EngineError as ex:
        err = f"{type(ex).__name__}: {ex}"
    dt = time.monotonic() - t0
    again = e.generate_ids(PROMPT, 200, temperature=0.0, stop_on_eos=False)
    torch.cuda.synchronize()
    return err, dt, streamed, long_ref, again == long_ref and not tp.custom_timed_out()


def _long_prefill(e, ref):
    """Work queued behind the prefill on the engine's stream takes ~4x the host's replay deadline:
    the decode must wait for it (not abort the collectives / break the group) and match ``ref``.
    -> (tokens match, group not broken, deadline s, queued work s)."""
    from llm_consensus_amd import ops

    x = torch.randn(4096, 4096, device=e.device).to(torch.bfloat16)
    y = torch.empty_like(x)

    def busy(n):
        with e._on_stream():
            for _ in range(n):
                ops.linear(x, x, ops.EPI_BF16, out=y)

    busy(2)
    e.stream.synchronize()
    t0 = time.monotonic()
    busy(20)
    e.stream.synchronize()
    per = (time.monotonic() - t0) / 20
    n = max(20, int(0.8 / per))  # ~0.8 s of queued work
    e.stall_s = 0.2
    orig = e.prefill

    def prefill(*a, **k):
        orig(*a, **k)
        busy(n)

    e.prefill = prefill
    toks = e.generate_ids(PROMPT, 24, temperature=0.0, stop_on_eos=False)
    torch.cuda.synchronize()
    return toks == ref, e.tp.broken is None, e.stall_s, n * per


def _run(layout, case="dead"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, layout, q, case)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=300) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


def _check(res):
    (_, e0, dt0, same0, checks0, tmo0), (_, e1, dt1, same1, checks1, tmo1) = res
    assert e1 and e1.startswith("InjectedEngineFault"), res
    assert e0 and "TP peer failed mid-decode" in e0, res
    # the survivor's replay waited on rank 1's collectives: its spins gave up (1-s bound) and the
    # agreed check re-synchronised the group (False = a timeout was found and resynced)
    assert checks0[:1] == [False] and checks1[:1] == [False], res
    assert dt0 < 10 and dt1 < 10, res
    assert same0 and same1, res
    assert not tmo0 and not tmo1, res


def test_tp_rank_stopping_mid_decode_fails_fast_cu_split(cuda):
    _check(_run("cu_split"))


def test_tp_rank_stopping_mid_decode_fails_fast_across_devices():
    if not torch.cuda.is_available() or torch.cuda.device_count() < 2:
        pytest.skip(f"needs 2 GPUs, this box has {torch.cuda.device_count()}")
    _check(_run("devices"))


def test_tp_rank_stalling_past_the_spin_bound_fails_before_streaming_stale_tokens(cuda):
    res = _run("cu_split", "stall")
    for rank, err, dt, streamed, long_ref, again_ok in res:
        assert err and err.startswith("EngineError"), res
        assert dt < 15, (rank, dt)
        # tokens up to the give-up are the clean run's; none computed after it reached the client
        assert len(streamed) <= 105 and streamed == long_ref[:len(streamed)], (rank, len(streamed))
        assert again_ok, rank


def test_tp_prefill_longer_than_the_replay_deadline_is_not_a_stall(cuda):
    res = _run("cu_split", "long_prefill")
    for rank, same, not_broken, stall_s, work_s in res:
        assert work_s > 2 * stall_s, (rank, stall_s, work_s)
        assert same and not_broken, res
