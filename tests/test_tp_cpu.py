"""Tensor parallelism on CPU with gloo (SURVEY.md §4.2 "TP / distributed" (a)): a TP=2 engine
(column/row-parallel linears, residual-folded all-reduce, vocab-parallel lm_head + all-gather,
sharded MoE experts) must reproduce the TP=1 model's logits and greedy tokens."""

import os
import socket

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


def _worker(rank, world, port, name, q, ekw=None, prompt_len=24):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        from llm_consensus_amd.engine import Engine, EngineConfig
        from llm_consensus_amd.models.config import FAMILIES
        from llm_consensus_amd.parallel.comm import TPGroup

        cfg = FAMILIES[name]
        tp = TPGroup(dist.group.WORLD, rank, world)
        e = Engine(cfg, EngineConfig(device="cpu", max_context=128, seed=5, **(ekw or {})), tp=tp)
        p = [(i * 13) % 700 + 256 for i in range(prompt_len)]
        s = e.new_sequence()
        e.prefill([s], [p])
        logits = e.full_logits(s).clone().unsqueeze(0)
        e.free_sequence(s)
        gen = e.generate_ids(p, 6, temperature=0.0, stop_on_eos=False)
        if rank == 0:
            q.put((logits.tolist(), gen))  # plain lists: tensor handles die with the child
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["llama-tiny", "mixtral-tiny", "phi3-tiny"])
def test_tp2_matches_tp1(name):
    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.models.config import FAMILIES

    ref = Engine(FAMILIES[name], EngineConfig(device="cpu", max_context=128, seed=5))
    p = [(i * 13) % 700 + 256 for i in range(24)]
    s = ref.new_sequence()
    ref.prefill([s], [p])
    ref_logits = ref.full_logits(s).clone()
    ref.free_sequence(s)
    ref_gen = ref.generate_ids(p, 6, temperature=0.0, stop_on_eos=False)

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, name, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    for pr in procs:
        if pr.is_alive():
            pr.kill()
            pr.join()
    assert all(pr.exitcode == 0 for pr in procs), [pr.exitcode for pr in procs]
    logits, gen = q.get(timeout=10)
    logits = torch.tensor(logits)
    # TP sums partials in a different order (and rounds partials to bf16): small drift only
    assert (logits[0] - ref_logits).abs().max().item() < 0.05 * ref_logits.abs().max().item()
    top2 = torch.topk(ref_logits, 2).values
    if (top2[0] - top2[1]).item() > 0.05:
        assert gen[0] == ref_gen[0]


def _run_tp(name, world, ekw, prompt_len):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q, ekw, prompt_len)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    for pr in procs:
        if pr.is_alive():
            pr.kill()
            pr.join()
    assert all(pr.exitcode == 0 for pr in procs), [pr.exitcode for pr in procs]
    logits, gen = q.get(timeout=10)
    return torch.tensor(logits)[0], gen


@pytest.mark.parametrize("name,ekw", [
    ("llama-tiny", {"sp_min_tokens": 8}),                                   # sequence parallel prefill
    ("mixtral-tiny", {"sp_min_tokens": 8}),                                 # SP + TP-sharded experts
    ("mixtral-tiny", {"expert_parallel": True, "sequence_parallel": False}),  # EP, replicated tokens
    ("mixtral-tiny", {"expert_parallel": True, "sp_min_tokens": 8}),        # EP + SP: all-to-all
])
def test_sp_ep_match_tp1(name, ekw):
    """Megatron sequence parallelism (reduce-scatter / all-gather around the norms, a ragged 25-token
    prompt padded to the shard size) and expert parallelism (whole experts per rank; all-to-all
    token dispatch under SP) reproduce the TP=1 model (SURVEY.md §2.5 SP / EP rows, C4)."""
    from llm_consensus_amd.engine import Engine, EngineConfig
    from llm_consensus_amd.models.config import FAMILIES

    ref = Engine(FAMILIES[name], EngineConfig(device="cpu", max_context=128, seed=5))
    p = [(i * 13) % 700 + 256 for i in range(25)]
    s = ref.new_sequence()
    ref.prefill([s], [p])
    ref_logits = ref.full_logits(s).clone()
    ref.free_sequence(s)
    ref_gen = ref.generate_ids(p, 6, temperature=0.0, stop_on_eos=False)
    logits, gen = _run_tp(name, 2, ekw, 25)
    assert (logits - ref_logits).abs().max().item() < 0.05 * ref_logits.abs().max().item()
    top2 = torch.topk(ref_logits, 2).values
    if (top2[0] - top2[1]).item() > 0.05:
        assert gen[0] == ref_gen[0]


class _FakeCarKernels:
    """Stand-in for the HIP module: mapping succeeds or fails per rank, and the all-reduce
    writes the right sum only where told to (exercises the group agreement, not the kernel)."""

    def __init__(self, rank, fail_open_rank=-1, correct_ranks=(), fail_alloc_rank=-1, timeout_rank=-1):
        self.rank, self.fail_open_rank, self.correct = rank, fail_open_rank, set(correct_ranks)
        self.fail_alloc_rank, self.timeout_rank = fail_alloc_rank, timeout_rank

    def car_alloc(self, cap):
        if self.rank == self.fail_alloc_rank:
            raise RuntimeError("car_alloc: out of memory")
        return 4096 * (self.rank + 1)

    def ipc_handle(self, p):
        return bytes([self.rank]) * 64

    def ipc_open(self, h):
        if self.rank == self.fail_open_rank:
            raise RuntimeError("ipc_open: invalid argument")
        return 1 << 20

    def ipc_close(self, p):
        pass

    def car_free(self, p):
        pass

    def car_timed_out(self, own):
        return 1 if self.rank == self.timeout_rank else 0

    def car_oneshot_max(self, cap):  # as allreduce.hip's car_oneshot_max
        return min(cap // 8 // 8 // 1024, 64) * 256 * 16

    def car_allreduce(self, bases, host, rank, world, cap, ptr, nbytes, stream):
        import ctypes

        if rank in self.correct:
            want = torch.full((nbytes // 2,), float(world * (world + 1) // 2), dtype=torch.bfloat16)
            ctypes.memmove(ptr, want.data_ptr(), nbytes)

    def car_twoshot(self, bases, host, rank, world, cap, mode, src, dst, seg_stride, seg16, nv, stream):
        assert mode == 0 and src == dst  # the self-test is an in-place all-reduce
        self.car_allreduce(bases, host, rank, world, cap, dst, nv * 16, stream)


def _car_agree_worker(rank, world, port, case, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import warnings

        from llm_consensus_amd.parallel import custom_ar
        from llm_consensus_amd.parallel.comm import TPGroup

        fake = {"open_fails": _FakeCarKernels(rank, fail_open_rank=1, correct_ranks=(0, 1)),
                "selftest_wrong": _FakeCarKernels(rank, correct_ranks=(0,)),
                "alloc_fails": _FakeCarKernels(rank, correct_ranks=(0, 1), fail_alloc_rank=1),
                "selftest_timeout": _FakeCarKernels(rank, correct_ranks=(0, 1), timeout_rank=1),
                "ok": _FakeCarKernels(rank, correct_ranks=(0, 1))}[case]
        custom_ar.kernels = lambda: fake
        tp = TPGroup(dist.group.WORLD, rank, world)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            enabled = tp.enable_custom(torch.device("cpu"))
        # the group is still in step afterwards: a plain collective gives the right answer
        t = torch.tensor([rank + 1.0])
        dist.all_reduce(t)
        q.put((rank, enabled, tp.custom is None, float(t.item())))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,want", [("open_fails", False), ("selftest_wrong", False), ("alloc_fails", False),
                                       ("selftest_timeout", False), ("ok", True)])
def test_custom_ar_enable_is_collective(case, want):
    """One rank failing to map a peer (or a self-test sum that is wrong on one rank) disables the
    custom all-reduce on EVERY rank, with no mismatched collectives: RCCL keeps the group."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_car_agree_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert len(r) == 4, r
        _, enabled, custom_none, tot = r
        assert enabled is want and custom_none is (not want) and tot == 3.0, r
