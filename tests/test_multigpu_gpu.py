"""Cross-device multi-GPU paths, one rank process per GPU (rank i on cuda:i, RCCL bootstrap), gated
on ``torch.cuda.device_count() >= N`` (skipped, not deselected, on a one-GPU box).

These are the paths a one-GPU box cannot execute and the driver's 8-GPU scaling run depends on
(reference fan-out ``internal/runner/runner.go:60-63``, judge ``internal/consensus/judge.go:96-99``):

* the custom xGMI collectives between distinct devices: ``hipDeviceCanAccessPeer``, cross-device
  ``hipIpcOpenMemHandle`` of the uncached buffers, one-shot all-reduce / all-gather and the two-shot
  reduce-scatter / all-gather / all-reduce, eagerly and replayed from a HIP graph;
* a TP = N engine's decode (custom collectives in its captured graphs) against TP = 1;
* ``bench.py --gpus N`` self-launched: the record must show N ranks on N distinct devices, the
  judge's custom all-reduce enabled and no spin timeout.
"""

import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLDS = [2, 4, 8]


def _need(n):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    have = torch.cuda.device_count()
    if have < n:
        pytest.skip(f"needs {n} GPUs, this box has {have}")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inp(rank, n, salt):
    g = torch.Generator().manual_seed(1000 * rank + n + salt)
    return torch.randn(n, generator=g).to(torch.bfloat16)


def _ar_exact(xs, times=1):
    """The custom collectives' result, bit for bit: f32 sum in rank order, rounded once to bf16, per
    in-place all-reduce (car_proto.h: every rank combines the granules in rank order)."""
    xs = [x.clone() for x in xs]
    for _ in range(times):
        acc = torch.zeros_like(xs[0], dtype=torch.float32)
        for x in xs:
            acc = acc + x.float()
        xs = [acc.to(torch.bfloat16)] * len(xs)
    return xs[0]


def _init(rank, world, port):
    import torch.distributed as dist

    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            device_id=torch.device("cuda", rank))
    return dist


def _run(target, world, *args, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=timeout) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


# ---- custom collectives across devices --------------------------------------------------------
def _collectives_worker(rank, world, port, q):
    try:
        dist = _init(rank, world, port)
        from llm_consensus_amd.parallel.comm import TPGroup
        from llm_consensus_amd.utils.native import kernels

        dev = f"cuda:{rank}"
        peers_ok = all(kernels().can_access_peer(rank, r) for r in range(world))
        tp = TPGroup(dist.group.WORLD, rank, world)
        enabled = tp.enable_custom(dev, cap=1 << 20, cap2=16 << 20)
        errs = []
        if enabled:
            for rep in range(2):
                for n in (8, 4096, 4104, 3 * 4096 + 8, 128 * 1024, 4 * (1 << 20) // 2 + 8 * 37):
                    x = _inp(rank, n, rep).to(dev)
                    tp.all_reduce_(x)  # one-shot up to 1 MiB, two-shot above
                    torch.cuda.synchronize()
                    errs.append(0.0 if torch.equal(x.cpu(), _ar_exact([_inp(r, n, rep) for r in range(world)])) else 1.0)
            loc = torch.full((2, 20), float(rank), dtype=torch.float32, device=dev)
            out = torch.empty(world, 2, 20, dtype=torch.float32, device=dev)
            tp.all_gather_rows(loc, out)
            Ts, H = 700, 4096
            full = _inp(rank, world * Ts * H, 7).view(world * Ts, H)
            rs = torch.empty(Ts, H, dtype=torch.bfloat16, device=dev)
            tp.reduce_scatter_rows(full.to(dev), rs)
            torch.cuda.synchronize()
            gather_ok = all(bool((out[r] == r).all()) for r in range(world))
            ref = _ar_exact([_inp(r, world * Ts * H, 7).view(world * Ts, H) for r in range(world)])[rank * Ts:(rank + 1) * Ts]
            errs.append(0.0 if torch.equal(rs.cpu(), ref) else 1.0)
            # graph replay with refreshed inputs (the decode graphs' pattern)
            n = 8192
            x = torch.zeros(n, dtype=torch.bfloat16, device=dev)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                tp.all_reduce_(x)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(3):
                    tp.all_reduce_(x)
            for rep in range(4):
                x.copy_(_inp(rank, n, 50 + rep))
                torch.cuda.synchronize()
                dist.barrier()
                g.replay()
                torch.cuda.synchronize()
                ref = _ar_exact([_inp(r, n, 50 + rep) for r in range(world)], times=3)  # three in-place
                errs.append(0.0 if torch.equal(x.cpu(), ref) else 1.0)
        else:
            gather_ok = False
        q.put((rank, peers_ok, enabled, max(errs) if errs else 1.0, gather_ok, tp.custom_timed_out() if enabled else None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, False, False, repr(e) + traceback.format_exc(), False, True))


@pytest.mark.parametrize("world", WORLDS)
def test_custom_collectives_across_devices(world):
    _need(world)
    for rank, peers_ok, enabled, err, gather_ok, tmo in _run(_collectives_worker, world):
        assert not isinstance(err, str), err
        assert peers_ok, f"rank {rank}: hipDeviceCanAccessPeer is false for a peer"
        assert enabled, f"rank {rank}: custom collectives fell back to RCCL"
        assert not tmo, f"rank {rank}: a custom-collective spin timed out"
        # every sum is the f32 rank-order sum rounded to bf16, bit for bit (a torn or stale granule
        # over xGMI would show here, where a tolerance would pass it)
        assert err == 0.0, f"rank {rank}: a cross-device sum differs from the f32 rank-order sum rounded to bf16"
        assert gather_ok, rank


# ---- TP decode across devices ----------------------------------------------------------------
def _tp_cfg():
    from llm_consensus_amd.models.config import ModelConfig

    # every sharded dimension divisible by 8: 16 heads, 8 kv heads, FFN 2048, vocab 32000
    return ModelConfig("llama-tp8-test", "llama", 2, 1024, 16, 8, 64, 2048, 32000, 500000.0, max_position=4096)


PROMPT = [(i * 13) % 700 + 256 for i in range(60)]


def _tp_worker(rank, world, port, q, layout="devices"):
    """A TP = world engine: ``devices`` = rank i on cuda:i over RCCL; ``one_gpu`` = every rank on
    cuda:0, each on its own 256 / world CUs (EngineConfig.cu_mask) with the fused row-parallel
    all-reduce forced on — the rehearsal the cross-device run must reproduce bit for bit."""
    try:
        if layout == "one_gpu":
            import torch.distributed as dist

            n = 256 // world
            os.environ["LLMC_CU_MASK"] = f"{rank * n}-{rank * n + n - 1}"
            os.environ["LLMC_FUSED_AR"] = "force"
            torch.cuda.set_device(0)
            dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
            dev = "cuda:0"
        else:
            dist = _init(rank, world, port)
            dev = f"cuda:{rank}"
        from llm_consensus_amd.engine import Engine, EngineConfig
        from llm_consensus_amd.parallel.comm import TPGroup

        ctrl = dist.new_group(list(range(world)), backend="gloo")
        tp = TPGroup(dist.group.WORLD, rank, world, ctrl=ctrl)
        enabled = tp.enable_custom(dev)
        e = Engine(_tp_cfg(), EngineConfig(device=dev, max_context=1024, seed=5), tp=tp)
        e.warmup_graphs()
        s = e.new_sequence()
        e.prefill([s], [PROMPT])
        logits = e.full_logits(s).float().cpu()
        e.free_sequence(s)
        gen = e.generate_ids(PROMPT, 32, temperature=0.0, stop_on_eos=False)
        torch.cuda.synchronize()
        q.put((rank, enabled and tp.custom_fused is not None, logits.tolist() if rank == 0 else None, gen,
               tp.custom_timed_out()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # noqa: BLE001
        import traceback

        q.put((rank, False, repr(ex) + traceback.format_exc(), None, True))


@pytest.mark.parametrize("world", WORLDS)
def test_tp_decode_across_devices_matches_tp1(world):
    _need(world)
    from llm_consensus_amd.engine import Engine, EngineConfig

    ref = Engine(_tp_cfg(), EngineConfig(device="cuda:0", max_context=1024, seed=5))
    s = ref.new_sequence()
    ref.prefill([s], [PROMPT])
    ref_logits = ref.full_logits(s).float().cpu()
    ref.free_sequence(s)
    ref_gen = ref.generate_ids(PROMPT, 32, temperature=0.0, stop_on_eos=False)
    del ref
    torch.cuda.empty_cache()
    res = _run(_tp_worker, world)
    gens = {}
    for rank, enabled, logits, gen, tmo in res:
        assert not isinstance(logits, str), logits
        assert enabled, f"rank {rank}: custom collectives (or the fused row-parallel all-reduce) fell back"
        assert not tmo, f"rank {rank}: a custom-collective spin timed out"
        gens[rank] = gen
        if rank == 0:
            lg = torch.tensor(logits)
            assert (lg - ref_logits).abs().max().item() < 0.05 * ref_logits.abs().max().item()
    assert all(g == gens[0] for g in gens.values()), "TP ranks sampled different tokens"
    agree = next((i for i, (a, b) in enumerate(zip(gens[0], ref_gen)) if a != b), len(ref_gen))
    assert agree >= 8, (agree, gens[0], ref_gen)  # bf16 sums in a different order: near-ties only late


@pytest.mark.parametrize("world", WORLDS)
def test_tp_decode_across_devices_bit_identical_to_one_gpu_rehearsal(world):
    """The same TP = N computation on N distinct devices (xGMI, RCCL bootstrap) and rehearsed on ONE
    GPU with CU-partitioned ranks: the push protocol sums in rank order (car_proto.h), so the
    prefill logits and the 32 greedy tokens must be bit-identical — a torn 8-byte granule or a stale
    epoch over the link would break this where a tolerance against TP = 1 would not."""
    _need(world)
    one = {r[0]: r for r in _run(_tp_worker, world, "one_gpu")}
    dev = {r[0]: r for r in _run(_tp_worker, world, "devices")}
    for res in (one, dev):
        for rank, enabled, logits, gen, tmo in res.values():
            assert not isinstance(logits, str), logits
            assert enabled and not tmo, rank
    assert torch.equal(torch.tensor(one[0][2]), torch.tensor(dev[0][2])), "prefill logits differ across layouts"
    assert all(one[r][3] == dev[r][3] for r in range(world)), (one[0][3], dev[0][3])


# ---- the bench's own multi-GPU flow ---------------------------------------------------------
@pytest.mark.parametrize("world", WORLDS)
def test_bench_self_launch_across_devices(world):
    _need(world)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(world), "--shapes", "tiny", "--steps", "1",
                        "--warmup", "0", "--max-tokens", "32", "--results-dir", ""],
                       cwd=ROOT, capture_output=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    d = json.loads([ln for ln in r.stdout.decode().splitlines() if ln.startswith("{")][0])
    x = d["extra"]
    assert d["n_gpus"] == world and x["dist_world_size"] == world
    assert [rd["device"] for rd in x["rank_devices"]] == list(range(world))
    assert len({rd["pci_bus_id"] for rd in x["rank_devices"]}) == world
    assert len(x["peer_access"]) >= world and all(x["peer_access"][i][j] for i in range(world) for j in range(world))
    judge = [k for k in x["custom_allreduce"] if k.endswith("@judge")]
    assert judge and x["custom_allreduce"][judge[0]] and not any(x["custom_allreduce_timed_out"].values())
    assert x["fused_rowparallel_allreduce"][judge[0]]
    assert x["allreduce_16k"][judge[0]]["impl"] == "custom_oneshot" and x["allreduce_16k"][judge[0]]["us"] > 0
    waits = x["collective_max_wait_us"][judge[0]]
    assert set(waits) >= {"oneshot", "fused"} and all(0 <= v < 1e6 for v in waits.values()), waits


@pytest.mark.parametrize("world", [2, 4])
def test_tp_one_gpu_rehearsal_is_deterministic(cuda, world):
    """The reference side of the bit-identity test above, on one GPU: the CU-partitioned TP = N
    rehearsal (fused row-parallel all-reduce forced on) gives the same prefill logits and greedy
    tokens on every run (runs on a one-GPU box)."""
    a = {r[0]: r for r in _run(_tp_worker, world, "one_gpu")}
    b = {r[0]: r for r in _run(_tp_worker, world, "one_gpu")}
    for res in (a, b):
        for rank, enabled, logits, gen, tmo in res.values():
            assert not isinstance(logits, str), logits
            assert enabled and not tmo, rank
    assert torch.equal(torch.tensor(a[0][2]), torch.tensor(b[0][2]))
    assert all(a[r][3] == b[r][3] for r in range(world))
