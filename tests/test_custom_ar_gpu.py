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
