"""K13: custom all-reduce / reduce-scatter / all-gather over IPC-mapped peer buffers.

Each rank allocates one uncached device buffer (signals + two data parities, see
``csrc/kernels/allreduce.hip``), exports it with hipIpc, and maps every peer's buffer; a
collective is then ONE kernel that stages the local data, signals each peer over xGMI, waits for
theirs (bounded spin) and reads the peers' copies directly. No host involvement per call, so it
is capturable in the decode HIP graph.

Two buffer classes per TP group (``TPGroup.enable_custom``):
  * one-shot (decode: <= 256 KiB, e.g. a [B, H] hidden state or a vocab-shard logits gather): every
    rank pushes its whole message into every peer's buffer as data-tagged granules and reduces what
    its peers pushed — one one-way trip over the link, no flag or fence; the same exchange also
    runs inside the row-parallel decode GEMVs' epilogue (``gemv_allreduce``, its own buffer);
  * two-shot (prefill: > 1 MiB, sequence-parallel reduce-scatter / all-gather): reduce-scatter +
    all-gather phases inside one launch, each rank pulling only 1/world of every peer's message per
    phase over all of its xGMI links at once; messages larger than the buffer run as pieces.
Setup is collective and self-checking: a rank that cannot map a peer (no P2P access between the
devices, IPC failure) or whose self-test sum is wrong makes EVERY rank fall back to RCCL together.
"""

from __future__ import annotations

import contextlib
import os
from typing import List, Optional

import torch

from ..utils.native import kernels

# bytes per data parity. One-shot: 8 slots of 8-B granules carrying 4 B each -> cap / 16 of payload
# per rank (256 KiB: a [4, 8192] bf16 hidden row is 64 KiB, the TP=2 logits gather [1, 64128] f32 256 KiB)
DEFAULT_CAP = 4 << 20
FUSED_CAP = 1 << 20     # the row-parallel GEMVs' fused all-reduce (EPI_AR): 16 granules x 1024 blocks per slot
TWOSHOT_CAP = 64 << 20  # bytes per parity of the two-shot buffer (larger messages run in pieces)
MODE_AR, MODE_RS, MODE_AG = 0, 1, 2


def _on(device: torch.device):
    return torch.cuda.device(device) if device.type == "cuda" else contextlib.nullcontext()


class CustomAllReduceUnavailable(RuntimeError):
    """Raised on EVERY rank of the group when any rank could not map the peers or the self-test
    failed: the group agrees before anyone raises, so the callers fall back together (RCCL)."""


class CustomAllReduceTimeout(RuntimeError):
    """A bounded spin gave up (a peer stalled): the results of the collectives since the last
    check are invalid; ``resync()`` restores a consistent protocol state."""


class CustomAllReduce:
    def __init__(self, group, rank: int, world: int, device: torch.device, cap: int = DEFAULT_CAP,
                 selftest: bool = True):
        import torch.distributed as dist

        if world > 8:
            raise ValueError("custom all-reduce supports up to 8 ranks (one xGMI hop)")
        self.rank, self.world, self.cap = rank, world, int(cap)
        self.device = torch.device(device)
        self.group = group
        self.own = 0
        self.host = self.host_dev = 0  # host status page (car_proto.h kHost*): host / device address
        self.bases: List[int] = []
        self._opened: List[int] = []
        err: Optional[BaseException] = None
        mine = None
        k = None
        if self.cap < 16 * world or self.cap % 16:
            err = ValueError(f"custom all-reduce cap {self.cap} too small / not a multiple of 16")
        else:
            try:
                k = kernels()
                with _on(self.device):
                    self.own = k.car_alloc(self.cap)
                    if self.device.type == "cuda":
                        self.host, self.host_dev = k.car_host_alloc()
                        spin_s = float(os.environ.get("LLMC_CAR_SPIN_S", "0") or 0)
                        if spin_s > 0:  # the spin bound (car_proto.h kHostSpinTicks; default 1 s)
                            # ticks of the 100-MHz clock in a 32-bit word the binding takes as int: <= 21 s
                            k.car_host_set(self.host, k.car_host_word(2), int(min(max(spin_s, 0.01), 21.0) * 1e8))
                    if self.device.type == "cuda":
                        dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
                    else:
                        dev_index = -1  # CPU fakes in tests
                    mine = (k.ipc_handle(self.own), int(dev_index))
            except Exception as e:  # noqa: BLE001 - reported collectively below
                err = e
        # every rank reaches every collective below, whatever failed locally (no mismatched calls)
        peers: List[Optional[tuple]] = [None] * world
        dist.all_gather_object(peers, mine, group=group)
        if err is None and any(p is None for p in peers):
            err = RuntimeError("a peer could not export its buffer")
        if err is None:
            try:
                with _on(self.device):
                    my_dev = peers[rank][1]
                    for r, (h, d) in enumerate(peers):
                        if r == rank:
                            self.bases.append(self.own)
                            continue
                        # a node whose GPUs cannot map each other's memory fails over cleanly
                        if my_dev >= 0 and not k.can_access_peer(my_dev, d):
                            raise RuntimeError(f"device {my_dev} has no peer access to device {d} (rank {r})")
                        p = k.ipc_open(h)
                        self.bases.append(p)
                        self._opened.append(p)
            except Exception as e:  # noqa: BLE001
                err = e
        # every rank on a device of its own (the fused row-parallel all-reduce needs it, comm.py)
        devs = [p[1] for p in peers if p is not None]
        self.distinct_devices = len(devs) == world and len(set(devs)) == world and all(d >= 0 for d in devs)
        ok = self._agree(err is None)
        if ok and selftest:
            ok = self._agree(self._selftest())
            if not ok and err is None:
                err = RuntimeError("self-test all-reduce returned wrong values or timed out")
        if not ok:
            self.close()
            raise CustomAllReduceUnavailable(f"rank {rank}: {err!r}" if err else f"rank {rank}: a peer failed")
        dist.barrier(group=group)

    def agree(self, ok: bool) -> bool:
        """MIN over the group of a local success flag (collective)."""
        return self._agree(ok)

    def _agree(self, ok: bool) -> bool:
        """MIN over the group of a local success flag (nccl wants a device tensor, gloo a host one)."""
        import torch.distributed as dist

        dev = self.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        f = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(f, op=dist.ReduceOp.MIN, group=self.group)
        return bool(int(f.item()))

    def _selftest(self) -> bool:
        """One real collective through the mapped peers before anything depends on it: a wrong
        sum or a spin that gave up (peer writes not visible over the link) disables the path."""
        try:
            one = kernels().car_oneshot_max(self.cap) // 2 if self.cap <= DEFAULT_CAP else self.cap // 2
            n = max(8, min(8192, one) // 8 * 8)  # <= 16 KiB: the decode hidden state of an 8B model
            x = torch.full((n,), float(self.rank + 1), dtype=torch.bfloat16, device=self.device)
            if self.cap > DEFAULT_CAP:
                self.all_reduce_large_(x)
            else:
                self.all_reduce_(x)
            if x.is_cuda:
                torch.cuda.synchronize(self.device)
            want = self.world * (self.world + 1) // 2
            return bool((x == want).all().item()) and not self.timed_out()
        except Exception:  # noqa: BLE001
            return False

    def fits(self, nbytes: int) -> bool:
        """Does a one-shot all-reduce / all-gather of ``nbytes`` per rank fit this buffer?"""
        return nbytes % 16 == 0 and nbytes <= kernels().car_oneshot_max(self.cap)

    # -- fused into the row-parallel GEMV (decode o_proj / down_proj) -----------------------------
    def gemv_allreduce(self, x: torch.Tensor, W: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
        """h = sum over ranks of W_r . x_r, rank 0's term + h (the residual): one GEMV launch with
        the one-shot exchange in its epilogue (gemv_core.h EPI_AR). x [M <= 2, K], W [N, K], h [M, N]
        bf16; same bits as ``linear(EPI_RESADD / EPI_BF16)`` + ``all_reduce_``."""
        M, K = x.shape
        N = W.shape[0]
        kernels().gemv_ar(M, x.data_ptr(), x.stride(0), W.data_ptr(), h.data_ptr(), h.stride(0), N, K, self.bases,
                          self.host_dev, self.rank, self.world, self.cap, self._stream(h))
        return h

    @staticmethod
    def _stream(t: torch.Tensor) -> int:
        return torch.cuda.current_stream(t.device).cuda_stream if t.is_cuda else 0

    # -- one-shot (decode) ----------------------------------------------------------------------
    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place bf16 sum over the group (f32 accumulation in rank order: every rank gets the
        same bits)."""
        if t.dtype != torch.bfloat16 or not t.is_contiguous():
            raise TypeError("custom all-reduce: contiguous bf16 only")
        kernels().car_allreduce(self.bases, self.host_dev, self.rank, self.world, self.cap, t.data_ptr(), t.numel() * 2,
                                self._stream(t))
        return t

    def all_gather(self, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """out.view(world, -1)[r] = x of rank r (any dtype; x contiguous)."""
        nbytes = x.numel() * x.element_size()
        if out.numel() * out.element_size() != nbytes * self.world:
            raise ValueError("custom all-gather: out must hold world * x")
        kernels().car_allgather(self.bases, self.host_dev, self.rank, self.world, self.cap, x.data_ptr(), out.data_ptr(),
                                nbytes, self._stream(x))
        return out

    # -- two-shot (prefill) -----------------------------------------------------------------------
    def all_reduce_large_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place bf16 sum, two-shot, in pieces of at most ``cap`` bytes (a multiple of 16 B)."""
        if t.dtype != torch.bfloat16 or not t.is_contiguous() or (t.numel() * 2) % 16:
            raise TypeError("two-shot all-reduce: contiguous bf16, multiple of 16 bytes")
        k, st = kernels(), self._stream(t)
        total = t.numel() * 2
        piece = self.cap // (16 * self.world) * 16 * self.world
        for o in range(0, total, piece):
            nb = min(piece, total - o)
            nv = nb // 16
            seg16 = (nv + self.world - 1) // self.world
            p = t.data_ptr() + o
            k.car_twoshot(self.bases, self.host_dev, self.rank, self.world, self.cap, MODE_AR, p, p, seg16 * 16, seg16, nv,
                          st)
        return t

    def reduce_scatter(self, full: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """out = rows [rank * n, (rank + 1) * n) of the bf16 sum of ``full`` [world * n, ...]."""
        seg = out.numel() * 2
        if (full.dtype != torch.bfloat16 or out.dtype != torch.bfloat16 or not full.is_contiguous()
                or not out.is_contiguous() or full.numel() != out.numel() * self.world or seg % 16):
            raise TypeError("two-shot reduce-scatter: contiguous bf16 [world*n] -> [n], 16-byte rows blocks")
        k, st = kernels(), self._stream(out)
        piece = self.cap // (16 * self.world) * 16
        for o in range(0, seg, piece):
            nb = min(piece, seg - o)
            k.car_twoshot(self.bases, self.host_dev, self.rank, self.world, self.cap, MODE_RS, full.data_ptr() + o,
                          out.data_ptr() + o, seg, nb // 16, self.world * (nb // 16), st)
        return out

    def all_gather_large(self, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """out.view(world, -1)[r] = x of rank r (any dtype), two-shot pieces."""
        seg = x.numel() * x.element_size()
        if out.numel() * out.element_size() != seg * self.world or seg % 16 or not x.is_contiguous():
            raise ValueError("two-shot all-gather: out must hold world * x, 16-byte multiple")
        k, st = kernels(), self._stream(x)
        piece = self.cap // (16 * self.world) * 16
        for o in range(0, seg, piece):
            nb = min(piece, seg - o)
            k.car_twoshot(self.bases, self.host_dev, self.rank, self.world, self.cap, MODE_AG, x.data_ptr() + o,
                          out.data_ptr() + o, seg, nb // 16, self.world * (nb // 16), st)
        return out

    # -- fault handling ---------------------------------------------------------------------------
    def timed_out(self) -> bool:
        """Did a spin of this rank give up (or return without its data) since the last resync?
        The host status page answers without a GPU call; the device word after a sync."""
        k = kernels()
        if self.host and k.car_host_get(self.host, k.car_host_word(1)):
            return True
        return bool(k.car_timed_out(self.own))

    def host_timed_out(self) -> bool:
        """``timed_out`` from the host status page only: no GPU call, safe while the stream runs."""
        k = kernels()
        return bool(self.host and k.car_host_get(self.host, k.car_host_word(1)))

    def aborted(self) -> bool:
        """Did the host set this rank's abort word since the last resync (every later spin then
        gives up at once: the buffer needs a resync even if no spin was waiting at the time)?"""
        k = kernels()
        return bool(self.host and k.car_host_get(self.host, k.car_host_word(0)))

    def abort(self) -> None:
        """Make every spin of this rank give up at its next check (~100 us) instead of polling to
        its 1-s limit: the host's way out of a replay that overran its deadline (a TP peer stalled
        or died). Cleared by ``resync``."""
        if self.host:
            k = kernels()
            k.car_host_set(self.host, k.car_host_word(0), 1)

    def max_wait_us(self) -> float:
        """Longest wait any spin of this buffer recorded since the last resync, in us (device
        read: call after a sync)."""
        return kernels().car_max_wait(self.own) / 100.0 if self.own and self.device.type == "cuda" else 0.0

    def resync(self) -> None:
        """Collective: after a spin timeout, every rank drains its device, then the protocol state
        (epochs, flags, timeout word) is zeroed on every rank between two group barriers."""
        import torch.distributed as dist

        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)
        with _on(self.device):
            k = kernels()
            k.car_reset(self.own, self.cap)
            if self.host:
                k.car_host_set(self.host, k.car_host_word(0), 0)
                k.car_host_set(self.host, k.car_host_word(1), 0)
        dist.barrier(group=self.group)

    def close(self) -> None:
        if not self.own and not self._opened:
            return
        k = kernels()
        for p in self._opened:
            try:
                k.ipc_close(p)
            except Exception:  # noqa: BLE001
                pass
        self._opened = []
        if self.own:
            k.car_free(self.own)
            self.own = 0
        if self.host:
            k.car_host_free(self.host)
            self.host = self.host_dev = 0
