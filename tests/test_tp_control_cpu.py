"""TP control-plane agreement (CPU ranks, gloo): every rank of a TP group must take the same
control decisions, or its collectives desynchronise (one extra replay on one rank = every later
custom all-reduce pairs the wrong epochs).

* cancellation: rank 1's cancel arrives one step later than rank 0's (and, in a second case,
  never) — both ranks still run the same number of decode steps and both stop with the error;
* batching: concurrent requests straddle the leader's batching window with different arrival
  times on each rank — the follower batches exactly the leader's requests;
* a custom-collective timeout on one rank fails the request on every rank and re-synchronises."""

import os
import queue
import socket
import threading
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _LateCtx:
    """done() turns True on the n-th call (None: never)."""

    def __init__(self, n):
        self.n, self.calls = n, 0

    def done(self):
        self.calls += 1
        return self.n is not None and self.calls >= self.n

    def err(self):
        return "context canceled" if self.done() else None

    def check(self):
        pass


def _cancel_worker(rank, world, port, cancel_at, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        from llm_consensus_amd.context import ContextError
        from llm_consensus_amd.engine import Engine, EngineConfig
        from llm_consensus_amd.models.config import FAMILIES
        from llm_consensus_amd.parallel.comm import TPGroup

        tp = TPGroup(dist.group.WORLD, rank, world, ctrl=dist.group.WORLD)
        e = Engine(FAMILIES["llama-tiny"], EngineConfig(device="cpu", max_context=256, seed=5), tp=tp)
        steps = [0]
        orig = e._decode_step

        def counted(B, bucket=None):
            steps[0] += 1
            return orig(B, bucket)

        e._decode_step = counted
        p = [(i * 13) % 700 + 256 for i in range(16)]
        err = None
        try:
            e.generate_ids(p, 40, temperature=0.0, stop_on_eos=False, ctx=_LateCtx(cancel_at[rank]))
        except ContextError as ex:
            err = str(ex)
        # the group is still in step: a second request decodes to the end on both ranks
        toks = e.generate_ids(p, 6, temperature=0.0, stop_on_eos=False)
        q.put((rank, steps[0], err, toks))
        dist.barrier()
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put((rank, -1, repr(ex) + traceback.format_exc(), None))
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("cancel_at", [(5, 6), (5, None), (None, 3)])
def test_cancel_is_the_leaders_decision(cancel_at):
    res = _spawn(_cancel_worker, 2, cancel_at)
    assert all(r[1] >= 0 for r in res), res
    (_, s0, e0, t0), (_, s1, e1, t1) = res
    assert s0 == s1, f"ranks ran {s0} vs {s1} decode steps"
    if cancel_at[0] is None:  # only a follower cancelled: the leader decides to go on
        assert e0 is None and e1 is None
    else:
        assert e0 and e1, (e0, e1)
    assert t0 == t1 and len(t0) == 6


class _FakeTP:
    def __init__(self, rank):
        self.rank, self.size, self.ctrl = rank, 2, dist.group.WORLD

    @property
    def is_leader(self):
        return self.rank == 0

    def leader_decides(self, v, kind="value"):
        from llm_consensus_amd.parallel.comm import TPGroup

        return TPGroup.leader_decides(self, v, kind)

    def _ctrl_exchange(self, kind, vals):
        from llm_consensus_amd.parallel.comm import TPGroup

        return TPGroup._ctrl_exchange(self, kind, vals)


class _FakeEngine:
    def __init__(self, rank):
        from types import SimpleNamespace

        self.ecfg = SimpleNamespace(max_batch=4)
        self.tp = _FakeTP(rank)


def _batch_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from llm_consensus_amd.runtime import worker as W

        h = object.__new__(W._EngineHost)
        h.engine = _FakeEngine(rank)
        h.q = queue.Queue()
        h._stash = W._EMPTY
        # a 200 ms batching window (instead of the default 5 ms) so thread wake-up jitter on a
        # loaded host cannot move an arrival across it: the leader sees r2 inside its window and
        # r3 after it; the follower sees r2 only after 400 ms (it must still batch it) and r3 right
        # behind it (it must not)
        W.BATCH_WINDOW_S = 0.2
        late = {0: (0.020, 0.600), 1: (0.400, 0.410)}[rank]

        def feed():
            time.sleep(late[0])
            h.q.put(("gen", "r2"))
            time.sleep(late[1] - late[0])
            h.q.put(("gen", "r3"))

        threading.Thread(target=feed, daemon=True).start()
        batch = [it[1] for it in h._gather(("gen", "r1"), "gen")]
        nxt = h._stash[1] if h._stash is not W._EMPTY else h.q.get(timeout=5)[1]
        q.put((rank, batch, nxt))
        dist.barrier()
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put((rank, repr(ex) + traceback.format_exc(), None))
    finally:
        dist.destroy_process_group()


def test_batch_membership_is_the_leaders():
    res = _spawn(_batch_worker, 2)
    (_, b0, n0), (_, b1, n1) = res
    assert b0 == ["r1", "r2"], res
    assert b1 == b0 and n0 == n1 == "r3", res


def _timeout_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        from llm_consensus_amd.engine import Engine, EngineConfig, EngineError
        from llm_consensus_amd.models.config import FAMILIES
        from llm_consensus_amd.parallel.comm import TPGroup

        class _FakeCustom:
            def __init__(self):
                self.tmo = rank == 1  # a spin gave up on rank 1 only
                self.resyncs = 0

            def timed_out(self):
                return self.tmo

            def host_timed_out(self):
                return self.tmo

            def aborted(self):
                return False

            def resync(self):
                self.resyncs += 1
                self.tmo = False

        tp = TPGroup(dist.group.WORLD, rank, world, ctrl=dist.group.WORLD)
        e = Engine(FAMILIES["llama-tiny"], EngineConfig(device="cpu", max_context=128, seed=5), tp=tp)
        fc = _FakeCustom()
        tp.custom = fc  # only consulted by the control plane on CPU tensors
        p = [(i * 13) % 700 + 256 for i in range(12)]
        err = None
        try:
            e.generate_ids(p, 4, temperature=0.0, stop_on_eos=False)
        except EngineError as ex:
            err = str(ex)
        ok = e.generate_ids(p, 4, temperature=0.0, stop_on_eos=False)  # after the resync
        q.put((rank, err, fc.resyncs, ok))
        dist.barrier()
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put((rank, repr(ex) + traceback.format_exc(), -1, None))
    finally:
        dist.destroy_process_group()


def test_custom_timeout_fails_request_on_every_rank_then_resyncs():
    res = _spawn(_timeout_worker, 2)
    for rank, err, resyncs, ok in res:
        assert err and "timed out" in err, res
        assert resyncs == 1 and ok is not None and len(ok) == 4, res


def _desync_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from llm_consensus_amd.parallel.comm import ControlDesync, TPGroup

        tp = TPGroup(dist.group.WORLD, rank, world, ctrl=dist.group.WORLD)
        assert tp.leader_decides(3 if rank == 0 else 0, "batch") == 3
        # the follower left its decode early: it asks for the next batch size while the leader
        # is still broadcasting a per-replay stop flag
        try:
            got = tp.leader_decides(0, "stop" if rank == 0 else "batch")
            q.put((rank, "value", got))
        except ControlDesync as ex:
            q.put((rank, "desync", str(ex)))
    except Exception as ex:  # noqa: BLE001
        q.put((rank, "error", repr(ex)))
    finally:
        dist.destroy_process_group()


def test_control_decisions_of_different_kinds_never_pair_up():
    """Both sides of a mismatched control round see it (every decision is the same all-reduce)."""
    (_, k0, v0), (_, k1, v1) = _spawn(_desync_worker, 2)
    assert k0 == "desync" and "expected stop" in v0 and "a peer sent batch" in v0, (k0, v0)
    assert k1 == "desync" and "expected batch" in v1 and "a peer sent stop" in v1, (k1, v1)


def test_gather_failure_replies_to_the_request_it_was_gathering_for():
    """A TP engine host whose batch-size broadcast fails (a peer is gone) answers the request it
    was gathering for with an error and finishes it — not a previous batch's requests."""
    from types import SimpleNamespace

    from llm_consensus_amd.runtime import worker as W

    class BrokenTP:
        size, rank, is_leader, ctrl = 2, 0, True, object()

        def leader_decides(self, v, kind="value"):
            raise RuntimeError("peer gone")

    sent, finished = [], []
    eng = SimpleNamespace(ecfg=SimpleNamespace(max_batch=1), tp=BrokenTP())
    h = W._EngineHost("m", eng, sent.append, leader=True, on_finished=finished.append)
    h.q.put(("gen", W._Req("r7", [1, 2], None, None)))
    h.q.put(None)
    h.t.join(timeout=10)
    assert [m[:2] for m in sent] == [("error", "r7")] and "peer gone" in sent[0][2]
    assert finished == ["r7"]


def _fault_worker(rank, world, port, mode, q):
    """A TP=2 engine on CPU ranks whose rank 1 fails mid-decode: ``stop`` = its engine raises before
    a replay (it stops launching; the peer's collectives would wait on it), ``die`` = its process
    exits. The survivor's request must fail within seconds, on the agreed replay; after a ``stop``
    the group is still in step and the next request matches a clean run."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import datetime

    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    try:
        torch.set_num_threads(1)
        from llm_consensus_amd.engine import Engine, EngineConfig, EngineError
        from llm_consensus_amd.models.config import FAMILIES
        from llm_consensus_amd.parallel.comm import TPGroup

        tp = TPGroup(dist.group.WORLD, rank, world, ctrl=dist.group.WORLD)
        e = Engine(FAMILIES["llama-tiny"], EngineConfig(device="cpu", max_context=256, seed=5), tp=tp)
        p = [(i * 13) % 700 + 256 for i in range(16)]
        ref = e.generate_ids(p, 12, temperature=0.0, stop_on_eos=False)
        if rank == 1 and mode == "stop":
            e.fault_at = ("decode", 7)

        def die(ids):
            os._exit(9)  # abrupt: no cleanup, like a segfault or an OOM kill

        t0 = time.monotonic()
        err = None
        try:
            e.generate_ids(p, 40, temperature=0.0, stop_on_eos=False,
                           on_tokens=(die if (rank == 1 and mode == "die") else None))
        except EngineError as ex:
            err = f"{type(ex).__name__}: {ex}"
        dt = time.monotonic() - t0
        again = None
        try:
            again = e.generate_ids(p, 12, temperature=0.0, stop_on_eos=False)
        except EngineError as ex:
            again = f"{type(ex).__name__}: {ex}"
        q.put((rank, err, dt, again == ref if isinstance(again, list) else again))
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put((rank, repr(ex) + traceback.format_exc(), -1, None))
    finally:
        if mode != "die":
            dist.destroy_process_group()


def test_tp_peer_raising_mid_decode_fails_every_rank_then_group_recovers():
    res = _spawn(_fault_worker, 2, "stop")
    (_, e0, dt0, again0), (_, e1, dt1, again1) = res
    assert e1 and e1.startswith("InjectedEngineFault"), res
    assert e0 and "TP peer failed mid-decode" in e0, res
    assert dt0 < 10 and dt1 < 10, res
    assert again0 is True and again1 is True, res


def test_tp_peer_process_death_fails_the_survivor_fast():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_fault_worker, args=(r, 2, port, "die", q)) for r in range(2)]
    for p in ps:
        p.start()
    rank, err, dt, again = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
    assert rank == 0 and err and "TP group broken" in err, (rank, err, dt, again)
    assert dt < 10, dt
    assert isinstance(again, str) and "TP group broken" in again, again
