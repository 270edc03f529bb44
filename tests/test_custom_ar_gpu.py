"""K13 custom all-reduce / all-gather on ONE GPU: 2 and 4 rank processes share the card, each
owning its uncached IPC buffer and mapping the others' (the same code path as across xGMI
peers, minus the link). Checked against an f32 sum of every rank's input, eagerly and replayed
from a HIP graph with changing inputs."""

import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SIZES = [8, 4096, 4104, 3 * 4096 + 8, 128 * 1024]  # elements (bf16): sub-chunk, chunk multiples, ragged


def _inp(rank, n, salt):
    g = torch.Generator().manual_seed(1000 * rank + n + salt)
    return torch.randn(n, generator=g).to(torch.bfloat16)


def _ar_exact(xs, times=1):
    """What the custom collectives must return, bit for bit: every rank's bf16 input summed in f32
    in rank order (0 + x_0 + x_1 + ...), rounded once to bf16 (RNE) — ``times`` in-place
    all-reduces in a row (after the first, every rank holds the same values)."""
    xs = [x.clone() for x in xs]
    for _ in range(times):
        acc = torch.zeros_like(xs[0], dtype=torch.float32)
        for x in xs:
            acc = acc + x.float()
        xs = [acc.to(torch.bfloat16)] * len(xs)
    return xs[0]


def _worker(rank, world, port, q):
    try:
        import torch.distributed as dist

        from llm_consensus_amd.parallel.comm import TPGroup

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        tp = TPGroup(dist.group.WORLD, rank, world)
        tp.enable_custom("cuda:0", cap=1 << 20)
        errs = []
        for rep in range(3):
            for n in SIZES:
                x = _inp(rank, n, rep).cuda()
                tp.all_reduce_(x)
                torch.cuda.synchronize()
                ref = _ar_exact([_inp(r, n, rep) for r in range(world)])
                errs.append(0.0 if torch.equal(x.cpu(), ref) else 1.0)  # rank-order sums: bit-exact
        # all-gather of f32 rows
        loc = torch.full((2, 5 * 4), float(rank), dtype=torch.float32, device="cuda")
        out = torch.empty(world, 2, 20, dtype=torch.float32, device="cuda")
        tp.all_gather_rows(loc, out)
        torch.cuda.synchronize()
        gather_ok = all(bool((out[r] == r).all()) for r in range(world))
        # graph capture: two all-reduces per replay, inputs refreshed before each replay
        n = 4096 * 2
        x = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
        y = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            tp.all_reduce_(x)
            tp.all_reduce_(y)
        torch.cuda.synchronize()
        dist.barrier()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            tp.all_reduce_(x)
            tp.all_reduce_(y)
        dist.barrier()
        for rep in range(4):
            x.copy_(_inp(rank, n, 50 + rep))
            y.copy_(_inp(rank, n, 90 + rep))
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            rx = _ar_exact([_inp(r, n, 50 + rep) for r in range(world)])
            ry = _ar_exact([_inp(r, n, 90 + rep) for r in range(world)])
            errs.append(0.0 if torch.equal(x.cpu(), rx) else 1.0)
            errs.append(0.0 if torch.equal(y.cpu(), ry) else 1.0)
        q.put((rank, max(errs), gather_ok, tp.custom.timed_out()))
        dist.barrier()
        tp.custom.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, repr(e) + traceback.format_exc(), False, True))


@pytest.mark.parametrize("world", [2, 4])
def test_custom_allreduce_ipc(cuda, world):
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    env_keep = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    assert env_keep in (None, "0")
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, err, gather_ok, tmo in res:
        assert not isinstance(err, str), err
        assert not tmo, f"rank {rank}: a barrier spin timed out"
        assert err == 0.0, f"rank {rank}: a sum differs from the f32 rank-order sum rounded to bf16"
        assert gather_ok, rank


def _twoshot_worker(rank, world, port, q):
    """Two-shot all-reduce / reduce-scatter / all-gather (prefill-sized messages, run in pieces
    when larger than the buffer) against f32 sums of every rank's input."""
    try:
        import torch.distributed as dist

        from llm_consensus_amd.parallel.comm import TPGroup

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        tp = TPGroup(dist.group.WORLD, rank, world)
        # a 16 MiB two-shot buffer: the 64 MiB case runs as pieces
        assert tp.enable_custom("cuda:0", cap=1 << 20, cap2=16 << 20)
        errs = []
        for mib in (4, 64):
            n = mib * (1 << 20) // 2 + 8 * 37  # ragged: last segment shorter
            x = _inp(rank, n, mib).cuda()
            tp.all_reduce_(x)
            torch.cuda.synchronize()
            ref = _ar_exact([_inp(r, n, mib) for r in range(world)])
            errs.append(0.0 if torch.equal(x.cpu(), ref) else 1.0)
        # sequence-parallel shapes: [world * Ts, H] -> [Ts, H] and back
        Ts, H = 1500, 4096
        full = [(_inp(r, world * Ts * H, 7).view(world * Ts, H)) for r in range(world)]
        out = torch.empty(Ts, H, dtype=torch.bfloat16, device="cuda")
        tp.reduce_scatter_rows(full[rank].cuda(), out)
        torch.cuda.synchronize()
        ref = _ar_exact(full)[rank * Ts:(rank + 1) * Ts]
        errs.append(0.0 if torch.equal(out.cpu(), ref) else 1.0)
        mine = _inp(rank, Ts * H, 11).view(Ts, H).cuda()
        g = torch.empty(world, Ts, H, dtype=torch.bfloat16, device="cuda")
        tp.all_gather_rows(mine, g)
        torch.cuda.synchronize()
        gat_ok = all(bool(torch.equal(g[r].cpu(), _inp(r, Ts * H, 11).view(Ts, H))) for r in range(world))
        q.put((rank, max(errs), gat_ok, tp.custom_timed_out()))
        dist.barrier()
        tp.custom.close()
        tp.custom2.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, repr(e) + traceback.format_exc(), False, True))


@pytest.mark.parametrize("world", [2, 4])
def test_twoshot_collectives_ipc(cuda, world):
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_twoshot_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, err, gat_ok, tmo in res:
        assert not isinstance(err, str), err
        assert not tmo, f"rank {rank}: a spin timed out"
        assert err == 0.0, f"rank {rank}: a two-shot sum differs from the f32 rank-order sum rounded to bf16"
        assert gat_ok, rank


def _cancel_tp_worker(rank, world, port, q):
    """A TP=2 engine (custom one-shot collectives in captured decode graphs, gloo control group)
    whose ranks see the cancel one replay apart: both stop at the leader's replay, the protocol
    stays in step (no spin timeout) and the next request is bit-identical to a clean run."""
    try:
        import torch.distributed as dist

        from llm_consensus_amd.context import ContextError
        from llm_consensus_amd.engine import Engine, EngineConfig
        from llm_consensus_amd.models.config import FAMILIES
        from llm_consensus_amd.parallel.comm import TPGroup

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        tp = TPGroup(dist.group.WORLD, rank, world, ctrl=dist.group.WORLD)
        assert tp.enable_custom("cuda:0")
        e = Engine(FAMILIES["llama-small"], EngineConfig(device="cuda:0", max_context=512, seed=3), tp=tp)
        e.warmup_graphs()
        p = [(i * 131) % 30000 + 256 for i in range(40)]
        ref = e.generate_ids(p, 48, temperature=0.0, stop_on_eos=False)

        class Late:
            def __init__(self, n):
                self.n, self.calls = n, 0

            def done(self):
                self.calls += 1
                return self.calls >= self.n

            def err(self):
                return "context canceled"

        err = None
        try:
            e.generate_ids(p, 400, temperature=0.0, stop_on_eos=False, ctx=Late(3 + rank))
        except ContextError as ex:
            err = str(ex)
        again = e.generate_ids(p, 48, temperature=0.0, stop_on_eos=False)
        torch.cuda.synchronize()
        q.put((rank, err, again == ref, tp.custom_timed_out()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put((rank, repr(ex) + traceback.format_exc(), False, True))


def test_tp_cancel_mid_decode_keeps_protocol_in_step(cuda):
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cancel_tp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    for rank, err, same, tmo in res:
        assert err == "context canceled", (rank, err)
        assert same, f"rank {rank}: the request after the cancel differs from the clean run"
        assert not tmo, f"rank {rank}: a spin timed out"


def _fused_worker(rank, world, port, q):
    """Row-parallel GEMV with the all-reduce in its epilogue (EPI_AR) against the two-launch path
    (EPI_RESADD on rank 0 / EPI_BF16 elsewhere, then the one-shot all-reduce): bit-identical, for
    one and two tokens, short (4-wave) and long (16-wave, 512-block) outputs, eagerly and replayed
    from a HIP graph with fresh inputs (epochs and data parities advance across launches)."""
    try:
        import torch.distributed as dist

        from llm_consensus_amd import ops
        from llm_consensus_amd.ops import EPI_BF16, EPI_RESADD
        from llm_consensus_amd.parallel.comm import TPGroup

        import os

        os.environ["LLMC_FUSED_AR"] = "force"  # ranks share the GPU (see comm.py): grids below fit together
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        tp = TPGroup(dist.group.WORLD, rank, world)
        assert tp.enable_custom("cuda:0") and tp.custom_fused is not None
        assert not tp.custom.distinct_devices
        car = tp.custom_fused
        bad = []

        def case(M, N, K, salt):
            g = torch.Generator().manual_seed(77 * rank + salt)
            x = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
            W = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).cuda()
            h0 = torch.randn(M, N, generator=torch.Generator().manual_seed(salt)).to(torch.bfloat16).cuda()
            return x, W, h0

        # every rank's grid resident at once on the shared GPU (2 x 1024-thread blocks or 8 x 256 per
        # CU): 16-wave grids of N / 16 blocks, 4-wave grids of N / 4 below N = 2048
        shapes = [(1, 2048, 512), (1, 2048, 1792), (2, 2048, 512), (1, 1024, 256), (2, 1536, 384)]
        if world == 2:
            shapes += [(1, 4096, 512), (2, 4096, 1792)]
        for M, N, K in shapes:
            for rep in range(3):
                x, W, h0 = case(M, N, K, 1000 * rep + N + K + M)
                hf = h0.clone()
                car.gemv_allreduce(x, W, hf)
                hr = h0.clone()
                ops.linear(x, W, EPI_RESADD if rank == 0 else EPI_BF16, out=hr)
                tp.all_reduce_(hr)
                torch.cuda.synchronize()
                if not torch.equal(hf, hr):
                    bad.append((M, N, K, rep, float((hf.float() - hr.float()).abs().max())))
        # graph: o-like then down-like fused launches per replay, inputs refreshed in place
        x1, W1, h = case(1, 2048, 512, 5)
        x2, W2, _ = case(1, 2048, 1792, 6)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            car.gemv_allreduce(x1, W1, h)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            car.gemv_allreduce(x1, W1, h)
            car.gemv_allreduce(x2, W2, h)
        for rep in range(4):
            xa, _, h0 = case(1, 2048, 512, 50 + rep)
            xb, _, _ = case(1, 2048, 1792, 90 + rep)
            x1.copy_(xa)
            x2.copy_(xb)
            h.copy_(h0)
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            hr = h0.clone()
            ops.linear(x1, W1, EPI_RESADD if rank == 0 else EPI_BF16, out=hr)
            tp.all_reduce_(hr)
            ops.linear(x2, W2, EPI_RESADD if rank == 0 else EPI_BF16, out=hr)
            tp.all_reduce_(hr)
            torch.cuda.synchronize()
            if not torch.equal(h, hr):
                bad.append(("graph", rep, float((h.float() - hr.float()).abs().max())))
        q.put((rank, bad, tp.custom_timed_out()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, repr(e) + traceback.format_exc(), True))


@pytest.mark.parametrize("world", [2, 4])
def test_fused_rowparallel_gemv_allreduce(cuda, world):
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fused_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, bad, tmo in res:
        assert not isinstance(bad, str), bad
        assert not tmo, f"rank {rank}: a spin timed out"
        assert bad == [], (rank, bad)
