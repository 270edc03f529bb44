"""K13: custom one-shot all-reduce / all-gather for decode-sized TP collectives.

Each rank allocates one uncached device buffer (signals + two data parities, see
``csrc/kernels/allreduce.hip``), exports it with hipIpc, and maps every peer's buffer; the
collective is then ONE kernel that stages the local slice, signals each peer over xGMI, waits
for theirs (bounded spin) and reads every peer's copy directly. No host involvement per call, so
it is capturable in the decode HIP graph (RCCL is used for bootstrap and for messages larger
than the buffer).
"""

from __future__ import annotations

import contextlib
from typing import List, Optional

import torch

from ..utils.native import kernels

DEFAULT_CAP = 1 << 20  # bytes per parity: [4, 8192] bf16 hidden = 64 KiB; logits gather [4, 32064] f32 = 512 KiB


def _on(device: torch.device):
    return torch.cuda.device(device) if device.type == "cuda" else contextlib.nullcontext()


class CustomAllReduceUnavailable(RuntimeError):
    """Raised on EVERY rank of the group when any rank could not map the peers or the self-test
    failed: the group agrees before anyone raises, so the callers fall back together (RCCL)."""


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
        self.bases: List[int] = []
        self._opened: List[int] = []
        err: Optional[BaseException] = None
        handle: Optional[bytes] = None
        k = None
        try:
            k = kernels()
            with _on(self.device):
                self.own = k.car_alloc(self.cap)
                handle = k.ipc_handle(self.own)
        except Exception as e:  # noqa: BLE001 - reported collectively below
            err = e
        # every rank reaches every collective below, whatever failed locally (no mismatched calls)
        handles: List[Optional[bytes]] = [None] * world
        dist.all_gather_object(handles, handle, group=group)
        if err is None and any(h is None for h in handles):
            err = RuntimeError("a peer could not export its buffer")
        if err is None:
            try:
                with _on(self.device):
                    for r, h in enumerate(handles):
                        if r == rank:
                            self.bases.append(self.own)
                        else:
                            p = k.ipc_open(h)
                            self.bases.append(p)
                            self._opened.append(p)
            except Exception as e:  # noqa: BLE001
                err = e
        ok = self._agree(err is None)
        if ok and selftest:
            ok = self._agree(self._selftest())
            if not ok and err is None:
                err = RuntimeError("self-test all-reduce returned wrong values or timed out")
        if not ok:
            self.close()
            raise CustomAllReduceUnavailable(f"rank {rank}: {err!r}" if err else f"rank {rank}: a peer failed")
        dist.barrier(group=group)

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
            n = 8192  # 16 KiB: the decode hidden state of an 8B model
            x = torch.full((n,), float(self.rank + 1), dtype=torch.bfloat16, device=self.device)
            self.all_reduce_(x)
            if x.is_cuda:
                torch.cuda.synchronize(self.device)
            want = self.world * (self.world + 1) // 2
            return bool((x == want).all().item()) and not self.timed_out()
        except Exception:  # noqa: BLE001
            return False

    def fits(self, nbytes: int) -> bool:
        return nbytes % 16 == 0 and nbytes <= self.cap

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place bf16 sum over the group (f32 accumulation in rank order: every rank gets the
        same bits)."""
        if t.dtype != torch.bfloat16 or not t.is_contiguous():
            raise TypeError("custom all-reduce: contiguous bf16 only")
        nbytes = t.numel() * 2
        stream = torch.cuda.current_stream(t.device).cuda_stream if t.is_cuda else 0
        kernels().car_allreduce(self.bases, self.rank, self.world, self.cap, t.data_ptr(), nbytes, stream)
        return t

    def all_gather(self, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """out.view(world, -1)[r] = x of rank r (any dtype; x contiguous)."""
        nbytes = x.numel() * x.element_size()
        if out.numel() * out.element_size() != nbytes * self.world:
            raise ValueError("custom all-gather: out must hold world * x")
        kernels().car_allgather(self.bases, self.rank, self.world, self.cap, x.data_ptr(), out.data_ptr(), nbytes,
                                torch.cuda.current_stream(x.device).cuda_stream)
        return out

    def timed_out(self) -> bool:
        return bool(kernels().car_timed_out(self.own))

    def rowpar_timed_out(self) -> bool:
        """Timeout word of a buffer used by gemv_rowpar_ar (its signal layout: ctr[1024] | flags
        [1024][8] | timeout at 36864; car_timed_out reads at the all-reduce layout's 3072)."""
        return bool(kernels().car_timed_out(self.own + (4 * 1024 + 1024 * 8 * 4) - (1024 + 64 * 8 * 4)))

    def gemv_rowpar_ar(self, x: torch.Tensor, W: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
        """Row-parallel decode projection with the all-reduce in the GEMV epilogue (EPI_AR):
        h = sum over ranks of x_r @ W_r^T, rank 0 folding the residual already in h. This
        object's buffer must be dedicated to it (block epochs of its own, cap >= 128 KiB)."""
        M, K = x.shape
        kernels().gemv_rowpar_ar(M, x.data_ptr(), x.stride(0), W.data_ptr(), h.data_ptr(), h.stride(0), W.shape[0], K,
                                 self.bases, self.rank, self.world, self.cap,
                                 torch.cuda.current_stream(x.device).cuda_stream)
        return h

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
