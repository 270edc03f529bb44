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
                ref = sum(_inp(r, n, rep).float() for r in range(world))
                errs.append(float((x.float().cpu() - ref).abs().max() / (ref.abs().max() + 1e-6)))
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
            rx = sum(_inp(r, n, 50 + rep).float() for r in range(world))
            ry = sum(_inp(r, n, 90 + rep).float() for r in range(world))
            errs.append(float((x.float().cpu() - rx).abs().max() / rx.abs().max()))
            errs.append(float((y.float().cpu() - ry).abs().max() / ry.abs().max()))
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
        assert err < 1e-2, (rank, err)
        assert gather_ok, rank


def _rowpar_worker(rank, world, port, q):
    """EPI_AR: the row-parallel GEMV with its all-reduce in the epilogue must give exactly the bits
    of GEMV (rank 0 residual-folded) + separate custom all-reduce, eagerly and from a HIP graph
    (1-2 rows; 3-4 rows within bf16 tolerance: the separate path's projection is the MFMA form)."""
    try:
        import torch.distributed as dist

        from llm_consensus_amd import ops
        from llm_consensus_amd.parallel.comm import TPGroup
        from llm_consensus_amd.parallel.custom_ar import CustomAllReduce

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        tp = TPGroup(dist.group.WORLD, rank, world)
        tp.enable_custom("cuda:0", cap=1 << 20)
        rp = CustomAllReduce(dist.group.WORLD, rank, world, "cuda:0", 128 * 1024, selftest=False)
        errs = []
        # per-rank grids stay small (<= 64 blocks): the ranks share this one GPU and every block of every
        # rank must be resident at once (on a node each rank has a GPU of its own)
        for M, N, K in [(1, 1024, 512), (2, 1024, 1792), (4, 1000, 256), (3, 1024, 1024)]:
            for rep in range(3):
                g = torch.Generator().manual_seed(7 * rank + rep + M * 1000 + K)
                x = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
                W = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16).cuda()
                g0 = torch.Generator().manual_seed(99 + rep + M)
                h0 = torch.randn(M, N, generator=g0).to(torch.bfloat16).cuda()  # same residual on all ranks
                ref = h0.clone()
                ops.linear(x, W, ops.EPI_RESADD if rank == 0 else ops.EPI_BF16, out=ref)
                tp.all_reduce_(ref)
                got = h0.clone()
                rp.gemv_rowpar_ar(x, W, got)
                torch.cuda.synchronize()
                if M <= 2:  # same VALU GEMV form on both sides: bit-exact
                    errs.append(int((got != ref).sum()))
                else:  # ops.linear takes the MFMA form from 3 rows on (EPI_AR stays on the VALU GEMV)
                    d = (got.float() - ref.float()).abs()
                    errs.append(int((d > 2e-2 + 2e-2 * ref.float().abs()).sum()))
        # graph replay with changing inputs
        M, N, K = 1, 1024, 512
        x = torch.zeros(M, K, dtype=torch.bfloat16, device="cuda")
        W = (torch.randn(N, K) * 0.05).to(torch.bfloat16).cuda()
        h = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            rp.gemv_rowpar_ar(x, W, h)
        torch.cuda.synchronize()
        dist.barrier()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            rp.gemv_rowpar_ar(x, W, h)
            rp.gemv_rowpar_ar(x, W, h)
        dist.barrier()
        for rep in range(3):
            x.copy_(torch.randn(M, K, generator=torch.Generator().manual_seed(rank * 31 + rep)).to(torch.bfloat16))
            h.copy_(torch.randn(M, N, generator=torch.Generator().manual_seed(500 + rep)).to(torch.bfloat16))
            ref = h.clone()
            for _ in range(2):
                ops.linear(x, W, ops.EPI_RESADD if rank == 0 else ops.EPI_BF16, out=ref)
                tp.all_reduce_(ref)
            torch.cuda.synchronize()
            dist.barrier()
            gr.replay()
            torch.cuda.synchronize()
            errs.append(int((h != ref).sum()))
        q.put((rank, max(errs) if max(errs) == 0 else str(errs), rp.rowpar_timed_out() or tp.custom.timed_out()))
        dist.barrier()
        rp.close()
        tp.custom.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, repr(e) + traceback.format_exc(), True))


@pytest.mark.parametrize("world", [2, 4])
def test_rowpar_fused_allreduce(cuda, world):
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rowpar_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, bad, tmo in res:
        assert not isinstance(bad, str), bad
        assert bad == 0, f"rank {rank}: {bad} elements differ from GEMV + separate all-reduce"
        assert not tmo, f"rank {rank}: a spin timed out"


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
            ref = sum(_inp(r, n, mib).float() for r in range(world))
            errs.append(float((x.float().cpu() - ref).abs().max() / ref.abs().max()))
        # sequence-parallel shapes: [world * Ts, H] -> [Ts, H] and back
        Ts, H = 1500, 4096
        full = [(_inp(r, world * Ts * H, 7).view(world * Ts, H)) for r in range(world)]
        out = torch.empty(Ts, H, dtype=torch.bfloat16, device="cuda")
        tp.reduce_scatter_rows(full[rank].cuda(), out)
        torch.cuda.synchronize()
        ref = sum(f.float() for f in full)[rank * Ts:(rank + 1) * Ts]
        errs.append(float((out.float().cpu() - ref).abs().max() / ref.abs().max()))
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
        assert err < 1e-2, (rank, err)
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
