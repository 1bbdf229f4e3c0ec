"""Collective transports of the distributed engine.

The distributed solve needs four collectives: all_gather (meta), all_to_all_single (counts and
the routing payload) and a MAX all-reduce (certification flag). Two backends provide them:

* ``TorchDistTransport`` -- ``torch.distributed`` (RCCL over xGMI with backend "nccl" on GPU
  ranks, gloo on CPU ranks). One process per GPU: the production path.
* ``LoopbackTransport``  -- N *virtual* ranks as threads of one process (one GPU or the CPU),
  exchanging tensors through a shared hub with barriers. Lets the whole multi-rank algorithm
  (decomposition, routing, halo certification, growth rounds) run and be checked bit-for-bit
  against the single-process oracle on a 1-GPU box. Ops of all virtual ranks go to the same
  device stream in barrier order, so cross-rank reads are stream-ordered after the writes.
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional

import torch
import torch.distributed as dist


class CollectiveError(RuntimeError):
    """A collective of the distributed engine failed or did not complete within the timeout
    (a peer rank died or hangs). The process should exit non-zero: the group is unusable."""


class TorchDistTransport:
    """``timeout_s``: failure detection inside the library, independent of the process group's
    own timeout. On a CPU backend (gloo) every collective is issued asynchronously and waited for
    at most that long. On RCCL ("nccl") collectives stay stream-ordered and never block the host:
    ``Work.wait(timeout)`` would make the CPU thread poll the collective to completion, which
    serialises the sync-free steady-state steps. A device-side hang or a dead peer is then caught
    by the group's watchdog (``TORCH_NCCL_ASYNC_ERROR_HANDLING``, on by default, aborts the
    process after the group's timeout); errors the call raises become ``CollectiveError``."""

    def __init__(self, group=None, timeout_s: Optional[float] = None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.timeout_s = timeout_s
        self.stream_ordered = dist.get_backend(group) == "nccl"

    def _run(self, name: str, fn):
        if self.timeout_s is None:
            fn(False)
            return
        if self.stream_ordered:
            try:
                fn(False)
            except Exception as e:  # noqa: BLE001 - report which collective and rank
                raise CollectiveError(f"rank {self.rank}: {name} failed: {e}") from e
            return
        import datetime

        try:
            work = fn(True)
            if work is not None and not work.wait(datetime.timedelta(seconds=self.timeout_s)):
                raise CollectiveError(f"rank {self.rank}: {name} did not complete within {self.timeout_s} s")
        except CollectiveError:
            raise
        except Exception as e:  # noqa: BLE001 - report which collective and rank
            raise CollectiveError(f"rank {self.rank}: {name} failed: {e}") from e

    def all_gather(self, t: torch.Tensor) -> List[torch.Tensor]:
        parts = [torch.empty_like(t) for _ in range(self.world)]
        self._run("all_gather", lambda a: dist.all_gather(parts, t, group=self.group, async_op=a))
        return parts

    def all_gather_cat(self, t: torch.Tensor) -> torch.Tensor:
        """All ranks' ``t`` concatenated (rank order), left on the device (no host sync)."""
        out = t.new_empty((self.world * t.numel(),))
        self._run("all_gather_into_tensor",
                  lambda a: dist.all_gather_into_tensor(out, t.contiguous().view(-1), group=self.group, async_op=a))
        return out

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None) -> None:
        self._run("all_to_all_single",
                  lambda a: dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group, async_op=a))

    def all_reduce_max(self, t: torch.Tensor) -> None:
        self._run("all_reduce", lambda a: dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group, async_op=a))


class HostStagedTransport(TorchDistTransport):
    """torch.distributed collectives on device tensors staged through host memory: lets a
    CPU-only backend (gloo) drive the GPU algorithm. Used to rehearse multi-PROCESS runs of the
    native path where RCCL cannot run them (several ranks on one GPU: "Duplicate GPU detected")."""

    def all_gather(self, t: torch.Tensor) -> List[torch.Tensor]:
        return [x.to(t.device) for x in super().all_gather(t.cpu())]

    def all_gather_cat(self, t: torch.Tensor) -> torch.Tensor:
        return super().all_gather_cat(t.cpu()).to(t.device)

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None) -> None:
        o = torch.empty(out.shape, dtype=out.dtype)
        super().all_to_all_single(o, inp.cpu(), out_splits, in_splits)
        out.copy_(o)

    def all_reduce_max(self, t: torch.Tensor) -> None:
        c = t.cpu()
        super().all_reduce_max(c)
        t.copy_(c)


class LoopbackHub:
    """Shared state of N virtual ranks (one per thread)."""

    def __init__(self, world: int, timeout: float = 300.0):
        self.world = world
        self.barrier = threading.Barrier(world, timeout=timeout)
        self.slots: list = [None] * world


class LoopbackTransport:
    def __init__(self, hub: LoopbackHub, rank: int):
        self.hub = hub
        self.rank = rank
        self.world = hub.world

    def _exchange(self, item):
        h = self.hub
        h.slots[self.rank] = item
        h.barrier.wait()
        got = list(h.slots)
        h.barrier.wait()  # nobody overwrites a slot before everyone has read it
        return got

    def all_gather(self, t: torch.Tensor) -> List[torch.Tensor]:
        return [x.clone() for x in self._exchange(t)]

    def all_gather_cat(self, t: torch.Tensor) -> torch.Tensor:
        return torch.cat([x.reshape(-1) for x in self._exchange(t)])

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None) -> None:
        n = inp.size(0)
        if in_splits is None:
            in_splits = [n // self.world] * self.world
        got = self._exchange((inp, list(in_splits)))
        parts = []
        for src_inp, src_splits in got:
            off = sum(src_splits[: self.rank])
            parts.append(src_inp[off:off + src_splits[self.rank]])
        if out.numel():
            torch.cat(parts, out=out)
        self.hub.barrier.wait()  # sources may free their send buffers only after the copies are enqueued

    def all_reduce_max(self, t: torch.Tensor) -> None:
        got = self._exchange(t.clone())
        r = got[0]
        for x in got[1:]:
            r = torch.maximum(r, x)
        t.copy_(r)


def run_loopback(world: int, fn: Callable[[LoopbackTransport], object], timeout: float = 300.0) -> list:
    """Run ``fn(transport)`` on ``world`` virtual ranks (threads); returns the per-rank results.
    An exception on any rank aborts the barrier for all and is re-raised."""
    hub = LoopbackHub(world, timeout)
    out: list = [None] * world
    err: list = [None]
    dev: Optional[int] = torch.cuda.current_device() if torch.cuda.is_available() else None

    def body(r: int):
        try:
            if dev is not None:
                torch.cuda.set_device(dev)
            out[r] = fn(LoopbackTransport(hub, r))
        except BaseException as e:  # noqa: BLE001 - propagate to the caller
            err[0] = err[0] or e
            hub.barrier.abort()

    ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout + 60)
    if err[0] is not None:
        raise err[0]
    return out
