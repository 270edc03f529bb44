"""Tensor-parallel communication.

One process per GPU; a TP group is a ``torch.distributed`` sub-group (backend "nccl" = RCCL over
xGMI on ROCm, "gloo" for CPU tests). The row-parallel reductions use the *residual-folding*
trick: rank 0 adds its partial product onto the residual stream, the other ranks write their
partial product into the same buffer, and ONE in-place all-reduce yields
``h + sum_r partial_r`` — no separate residual-add kernel and no extra buffer per layer.

On GPUs the collectives go through the custom xGMI kernels (``custom_ar.py``, K13) once
``enable_custom()`` has mapped the peers: one-shot for decode-sized messages (no RCCL call and no
host work per collective, so a TP engine's decode step is capturable in one HIP graph) and
two-shot (reduce-scatter + all-gather phases over peer reads) for prefill-sized ones. RCCL is the
fallback when a group cannot map its peers (its collectives are then captured in the decode graphs
too, after a collective self-check: ``graph_capture_ok``); CPU/gloo groups use torch.distributed.

Control plane: TP ranks must take every control decision identically (which requests form a
batch, when a decode stops on cancellation or deadline), or their collectives desynchronise. A
TP group therefore carries a host-side ``ctrl`` group (gloo) over the same ranks: the leader's
decisions (``leader_decides``) and the per-replay stop / failure / done vote of a decode
(``step_agree``) are the same sequence-checked all-reduce, and fault checks are agreed by all ranks
(``any_rank``). A failure anywhere in the group therefore ends the request on every rank at the same
replay; a peer that dies or stalls ends it within the custom collectives' 1-s spin bound plus one
control round (``ctrl_timeout`` for a stalled host).

Prefill under TP can run Megatron-style SEQUENCE PARALLEL (engine ``EngineConfig.sequence_parallel``):
the residual stream is sharded by token rows between the layers, so each row-parallel output is a
reduce-scatter (``reduce_scatter_rows``) and each norm runs on 1/tp of the tokens before an
all-gather (``all_gather_rows``) feeds the next column-parallel GEMM — the same bytes on xGMI as
the all-reduce, 1/tp of the norm/residual work and activation memory per rank. MoE models can
shard EXPERTS instead of their FFN rows (``EngineConfig.expert_parallel``); with sequence-parallel
token shards the tokens travel to their experts' ranks and back by all-to-all (``all_to_all_rows``).
"""

from __future__ import annotations

import warnings

from typing import List, Optional

import torch
import torch.distributed as dist


CTRL_KINDS = {"value": 1, "batch": 2, "stop": 3, "step": 4}


class ControlDesync(RuntimeError):
    """The TP ranks' control decisions no longer pair up (see ``TPGroup.leader_decides``)."""


class TPGroup:
    """Rank/size of a model's tensor-parallel group (size 1 = no communication)."""

    def __init__(self, group: Optional["dist.ProcessGroup"] = None, rank: int = 0, size: int = 1,
                 ctrl: Optional["dist.ProcessGroup"] = None):
        self.group = group
        self.rank = rank
        self.size = size
        self.ctrl = ctrl      # host control group (gloo) over the same ranks, or None
        # set when the group can no longer agree (a peer process died, a control round timed out,
        # or a device wait overran twice): every later request on its engines fails at once
        self.broken: Optional[str] = None
        self.custom = None    # one-shot CustomAllReduce once enable_custom() ran
        self.custom2 = None   # its two-shot twin for prefill-sized messages
        self.custom_fused = None  # the row-parallel decode GEMVs' fused all-reduce buffer (EPI_AR)

    def enable_custom(self, device, cap: Optional[int] = None, cap2: Optional[int] = None) -> bool:
        """Map the group's IPC buffers for the custom collectives (GPU groups of 2..8 ranks).
        Collective; returns False on every rank (RCCL stays in charge) when any rank failed."""
        if self.size == 1 or self.custom is not None:
            return self.custom is not None
        import os

        from .custom_ar import DEFAULT_CAP, FUSED_CAP, TWOSHOT_CAP, CustomAllReduce, CustomAllReduceUnavailable

        try:
            self.custom = CustomAllReduce(self.group, self.rank, self.size, device, cap or DEFAULT_CAP)
            self.custom2 = CustomAllReduce(self.group, self.rank, self.size, device, cap2 or TWOSHOT_CAP)
            # the same decision on every rank (environment of the whole job; A/B: LLMC_FUSED_AR=0).
            # Ranks sharing one GPU keep separate launches unless forced (LLMC_FUSED_AR=force: the
            # CU-partitioned rehearsals): a fused GEMV block spins on its peers' blocks of the SAME
            # launch, and two ranks' full-chip grids on one device can leave a peer's blocks
            # waiting for CUs the spinning blocks hold (on separate GPUs the lowest unfinished
            # block is always resident)
            fused = os.environ.get("LLMC_FUSED_AR", "1")
            if fused == "force" or (fused != "0" and self.custom.distinct_devices):
                # no one-shot self-test on this buffer: its granule layout is the fused GEMV's
                # (16 per block), and a one-shot kernel's granules (1024 per block) left in it would
                # carry tags that block's epochs reach again; the peers were just verified above
                self.custom_fused = CustomAllReduce(self.group, self.rank, self.size, device, FUSED_CAP,
                                                    selftest=False)
                if not self.custom.agree(self._fused_selftest(device)):
                    warnings.warn("fused row-parallel all-reduce failed its self-test: separate all-reduce launches")
                    # every rank's fused launches have drained (the self-test synchronised, also on
                    # its error path) before the agreement above, so no peer still writes into the
                    # buffer being closed; then the one-shot path restarts from a clean state
                    self.custom_fused.close()
                    self.custom_fused = None
                    self.custom.resync()
        except CustomAllReduceUnavailable as e:
            warnings.warn(f"custom all-reduce disabled, using RCCL: {e}")
            for c in (self.custom, self.custom2, self.custom_fused):
                if c is not None:
                    c.close()
            self.custom = self.custom2 = self.custom_fused = None
            return False
        return True

    def _fused_selftest(self, device) -> bool:
        """The fused row-parallel GEMV all-reduce (EPI_AR) against the same GEMV + the one-shot
        all-reduce just verified, bit for bit, over three launches (epochs and both data parities);
        any error or spin timeout is a failure. Collective (every rank runs it)."""
        try:
            from .. import ops

            dev = torch.device(device)
            g = torch.Generator().manual_seed(4242 + self.rank)
            ok = True
            for rep in range(3):
                x = torch.randn(1, 512, generator=g).to(torch.bfloat16).to(dev)
                W = (torch.randn(1024, 512, generator=g) / 16).to(torch.bfloat16).to(dev)
                h0 = torch.randn(1, 1024, generator=torch.Generator().manual_seed(rep)).to(torch.bfloat16).to(dev)
                hf = h0.clone()
                self.custom_fused.gemv_allreduce(x, W, hf)
                hr = h0.clone()
                ops.linear(x, W, ops.EPI_RESADD if self.rank == 0 else ops.EPI_BF16, out=hr)
                self.custom.all_reduce_(hr)
                if dev.type == "cuda":
                    torch.cuda.synchronize(dev)
                ok = ok and bool(torch.equal(hf, hr))
            return ok and not self.custom_fused.timed_out() and not self.custom.timed_out()
        except Exception:  # noqa: BLE001
            if torch.device(device).type == "cuda":
                try:  # whatever was launched finishes before the group decides (and closes buffers)
                    torch.cuda.synchronize(torch.device(device))
                except Exception:  # noqa: BLE001
                    pass
            return False

    def collectives(self):
        return [c for c in (self.custom, self.custom2, self.custom_fused) if c is not None]

    def graph_capture_ok(self, device) -> bool:
        """Can this group's RCCL collectives run inside the engine's decode HIP graphs? The
        fallback when the custom kernels are unavailable: instead of decoding eagerly (~320
        launches + 64 host-issued RCCL calls per token), capture RCCL too. Collective: every rank
        captures an all-reduce + all-gather, the group agrees before anyone replays (a rank that
        failed to capture never leaves peers waiting in a replayed collective), then checks the
        sums and agrees again. False on every rank if anything failed; gloo groups are never
        capturable."""
        if self.size == 1:
            return True
        if self.group is None or dist.get_backend(self.group) != "nccl":
            return False

        def agree(ok: bool) -> bool:  # MIN over the group, eager RCCL on a one-element tensor
            t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
            return bool(t.item())

        cap = rccl_graph_capture(self.group, self.rank, self.size, device)
        if not agree(cap is not None):
            return False
        return agree(rccl_graph_replay_check(cap, self.rank, self.size, device))

    # -- control plane ----------------------------------------------------------------------------
    def _ctrl_exchange(self, kind: str, vals: List[int]) -> List[int]:
        """One control round over ``ctrl``: every rank contributes (kind, sequence number, vals) and
        gets the element-wise MAX of ``vals``. Every control decision is this same collective (an
        all-reduce), so ranks whose call sequences shifted (one left a decode early) still meet in
        a matching collective and both see the mismatch: the kinds or sequence numbers differ, and
        ``ControlDesync`` is raised on every rank involved instead of one acting on a value meant
        for another decision. A peer process that died makes gloo raise at once; a stalled one,
        after the group's timeout (``ctrl_timeout``)."""
        code = CTRL_KINDS[kind]
        self._ctrl_seq = getattr(self, "_ctrl_seq", 0) + 1
        seq = self._ctrl_seq
        t = torch.tensor([code, -code, seq, -seq, *vals], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.ctrl)
        hi_k, lo_k, hi_s, lo_s = int(t[0]), -int(t[1]), int(t[2]), -int(t[3])
        if hi_k != code or lo_k != code or hi_s != seq or lo_s != seq:
            names = {v: k for k, v in CTRL_KINDS.items()}
            other = names.get(hi_k if hi_k != code else lo_k, hi_k)
            oseq = hi_s if hi_s != seq else lo_s
            raise ControlDesync(f"TP control channel out of step on rank {self.rank}: expected {kind} #{seq}, "
                                f"a peer sent {other} #{oseq}")
        return [int(v) for v in t[4:]]

    def leader_decides(self, value: int, kind: str = "value") -> int:
        """The leader's ``value`` (>= 0) on every rank; identity without a control group. A
        ``_ctrl_exchange`` in which only the leader's value counts (the followers send -1)."""
        if self.size == 1 or self.ctrl is None:
            return value
        return self._ctrl_exchange(kind, [int(value) if self.is_leader else -1])[0]

    def step_agree(self, stop: bool, failed: bool, done: bool):
        """Per-replay decision of a TP decode, one control round: (stop, failed, done) where stop =
        the LEADER's cancellation / deadline (a follower's own cancel arrives at its own time),
        failed = ANY rank's engine failed since the last round (its replays stopped, or its
        streaming raised), done = EVERY rank has all its rows finished. Every rank then leaves the
        decode at the same replay, so the collectives of the replays they did launch pair up."""
        if self.size == 1 or self.ctrl is None:
            return bool(stop), bool(failed), bool(done)
        lead = int(bool(stop)) if self.is_leader else 0
        st, fl, notdone = self._ctrl_exchange("step", [lead, int(bool(failed)), int(not done)])
        return bool(st), bool(fl), not notdone

    def any_rank(self, flag: bool) -> bool:
        """True on every rank if ``flag`` is True on any rank (host all-reduce over ``ctrl``)."""
        if self.size == 1 or self.ctrl is None:
            return bool(flag)
        t = torch.tensor([1 if flag else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.ctrl)
        return bool(t.item())

    def abort_collectives(self) -> None:
        """Local, no GPU call: every custom-collective spin of this rank gives up at its next check
        (a replay overran the host's deadline: a peer stalled or died). Cleared by a resync."""
        for c in self.collectives():
            c.abort()

    def resync_collectives(self) -> None:
        """Collective over the group: zero every custom collective's protocol state (epochs, flags,
        timeout words, wait statistics) between two barriers."""
        for c in self.collectives():
            c.resync()

    def collective_max_wait_us(self) -> dict:
        """Longest wait any spin recorded per collective buffer since the last resync, us (device
        reads: after a sync): one-shot (decode all-reduce / logits gather), two-shot (prefill),
        fused (the row-parallel GEMVs' epilogue)."""
        out = {}
        for name, c in (("oneshot", self.custom), ("twoshot", self.custom2), ("fused", self.custom_fused)):
            if c is not None:
                out[name] = round(c.max_wait_us(), 2)
        return out

    def custom_timed_out(self) -> bool:
        """Local: did a custom-collective spin give up, or the host abort this rank's spins, since
        the last resync (reads device memory, after the caller synchronised its stream)?"""
        return any(c.timed_out() or c.aborted() for c in self.collectives())

    def check_collectives(self) -> bool:
        """Collective over ``ctrl`` (every rank calls it at the same point): True when every rank's
        custom collectives completed; otherwise every rank re-synchronises the protocol state
        (epochs, flags) and False is returned everywhere, so the caller fails the work done since
        the last check instead of serving sums that read stale peer data."""
        if self.size == 1 or self.custom is None:
            return True
        if not self.any_rank(self.custom_timed_out()):
            return True
        for c in self.collectives():
            c.resync()
        return False

    @staticmethod
    def single() -> "TPGroup":
        return TPGroup(None, 0, 1)

    @staticmethod
    def from_group(group) -> "TPGroup":
        return TPGroup(group, dist.get_rank(group), dist.get_world_size(group))

    @property
    def is_leader(self) -> bool:
        return self.rank == 0

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.size > 1:
            c = self.custom
            nbytes = t.numel() * t.element_size()
            if c is not None and t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and nbytes % 16 == 0:
                return c.all_reduce_(t) if c.fits(nbytes) else self.custom2.all_reduce_large_(t)
            if self._bounce(t):
                f = t.cpu()
                dist.all_reduce(f, group=self.group)
                return t.copy_(f)
            dist.all_reduce(t, group=self.group)
        return t

    def all_gather_rows(self, t: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """Gather [B, n] shards into [size, B, n] (rank-major)."""
        if self.size == 1:
            out.view_as(t).copy_(t)
            return out
        c = self.custom
        nbytes = t.numel() * t.element_size()
        if c is not None and t.is_cuda and t.is_contiguous() and out.is_contiguous() and nbytes % 16 == 0:
            return c.all_gather(t, out) if c.fits(nbytes) else self.custom2.all_gather_large(t, out)
        flat = out.view(self.size * t.shape[0], *t.shape[1:])  # gloo wants dim-0 concatenation
        if self._bounce(t):
            f = flat.cpu()
            dist.all_gather_into_tensor(f, t.contiguous().cpu(), group=self.group)
            flat.copy_(f)
            return out
        dist.all_gather_into_tensor(flat, t.contiguous(), group=self.group)
        return out

    def _bounce(self, t: torch.Tensor) -> bool:
        """gloo collectives on GPU tensors (one-GPU rehearsals) go through host copies."""
        return t.is_cuda and dist.get_backend(self.group) != "nccl"

    def reduce_scatter_rows(self, full: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """Sum ``full`` [size * n, ...] over the group and keep this rank's row block
        ``out`` [n, ...] = rows [rank * n, (rank + 1) * n) (Megatron SP)."""
        if self.size == 1:
            return out.copy_(full)
        n = out.shape[0]
        c = self.custom2
        if (c is not None and full.is_cuda and full.dtype == torch.bfloat16 and full.is_contiguous()
                and out.is_contiguous() and (out.numel() * 2) % 16 == 0):
            return c.reduce_scatter(full, out)
        if full.is_cuda and not self._bounce(full):
            dist.reduce_scatter_tensor(out, full.contiguous(), group=self.group)
            return out
        # gloo has no reduce-scatter: all-reduce, then keep the local block (same result)
        f = full.cpu() if full.is_cuda else full
        dist.all_reduce(f, group=self.group)
        return out.copy_(f[self.rank * n:(self.rank + 1) * n])

    def exchange_counts(self, send_counts: List[int]) -> List[int]:
        """All-to-all of one int per peer: how many rows every peer will send me."""
        if self.size == 1:
            return list(send_counts)
        nccl = dist.get_backend(self.group) == "nccl"
        dev = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")
        s = torch.tensor(send_counts, dtype=torch.int64, device=dev)
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s, group=self.group)
        return [int(v) for v in r.tolist()]

    def all_to_all_rows(self, x: torch.Tensor, send_counts: List[int], recv_counts: List[int]) -> torch.Tensor:
        """Rows [sum(send_counts), ...] split by destination rank -> rows from every peer (C4,
        expert-parallel token dispatch/combine)."""
        out = x.new_empty((sum(recv_counts),) + tuple(x.shape[1:]))
        if self.size == 1:
            return out.copy_(x)
        if self._bounce(x):
            o = out.cpu()
            dist.all_to_all_single(o, x.contiguous().cpu(), output_split_sizes=recv_counts,
                                   input_split_sizes=send_counts, group=self.group)
            return out.copy_(o)
        dist.all_to_all_single(out, x.contiguous(), output_split_sizes=recv_counts, input_split_sizes=send_counts,
                               group=self.group)
        return out

    def broadcast_(self, t: torch.Tensor, src_rank_in_group: int = 0) -> torch.Tensor:
        if self.size > 1:
            src = dist.get_global_rank(self.group, src_rank_in_group) if self.group is not None else src_rank_in_group
            dist.broadcast(t, src=src, group=self.group)
        return t

    def barrier(self) -> None:
        if self.size > 1:
            dist.barrier(group=self.group)


def rccl_graph_capture(group, rank: int, size: int, device):
    """Capture an all-reduce and an all-gather of small fp32 buffers over ``group`` in one HIP
    graph (after an eager warm-up collective); (graph, x, y) or None if capture failed."""
    try:
        x = torch.full((256,), float(rank + 1), dtype=torch.float32, device=device)
        y = torch.empty(size * 256, dtype=torch.float32, device=device)
        dist.all_reduce(x.clone(), group=group)  # communicator ready before the capture
        torch.cuda.synchronize(device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=torch.cuda.Stream(device)):
            dist.all_reduce(x, group=group)
            dist.all_gather_into_tensor(y, x, group=group)
        return g, x, y
    except Exception as e:  # noqa: BLE001
        warnings.warn(f"RCCL graph capture failed ({type(e).__name__}: {e}); TP decode stays eager")
        return None


def rccl_graph_replay_check(cap, rank: int, size: int, device) -> bool:
    """Replay a ``rccl_graph_capture`` graph twice from fresh inputs and check the sums."""
    g, x, y = cap
    try:
        total = size * (size + 1) / 2
        for _ in range(2):
            x.fill_(float(rank + 1))
            g.replay()
        torch.cuda.synchronize(device)
        return bool((x == total).all()) and bool((y == total).all())
    except Exception as e:  # noqa: BLE001
        warnings.warn(f"RCCL graph replay failed ({type(e).__name__}: {e}); TP decode stays eager")
        return False


def shard_range(n: int, rank: int, size: int):
    if n % size != 0:
        raise ValueError(f"dimension {n} not divisible by tp={size}")
    s = n // size
    return rank * s, (rank + 1) * s
