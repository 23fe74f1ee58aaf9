"""SPMD distributed context: one process per GPU over ``torch.distributed``.

Replaces the reference's three data-parallel mechanisms — ``pmap`` +
``all_gather`` (``std_workflow.py:311-345``), GSPMD (``:253-309``) and the Ray
actor workflow (``workflows/distributed.py``) — with one MI355X-native model:
every rank holds a replica of the algorithm state, evaluates (or generates) a
balanced contiguous slice of the population, and exchanges only what is needed
through RCCL collectives over xGMI (backend ``"nccl"`` is RCCL on ROCm; ``gloo``
is used for CPU runs and tests).

Message sizes at the north-star shapes are small and latency-bound (fitness
slices of ≤ 40 KB, CMA-ES partial sums of 4 MB), so the context issues one
collective per exchange and never splits tensors into per-row messages.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..core.state import State, tree_flatten, tree_unflatten


def balanced_slices(n: int, world: int):
    """``[(start, size)]`` with the remainder spread over the first ranks
    (reference ``distributed.py:40-45``; fixes the dropped-remainder quirk of
    ``std_workflow.py:333``)."""
    q, r = divmod(n, world)
    out, start = [], 0
    for i in range(world):
        size = q + (1 if i < r else 0)
        out.append((start, size))
        start += size
    return out


class DistContext:
    def __init__(self, group=None, algorithm=None):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("torch.distributed is not initialised; call evoxmi.parallel.init_distributed() first")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.algorithm_sharded = algorithm is not None and hasattr(algorithm, "ask_sharded") and hasattr(algorithm, "tell_sharded")
        self.global_pop = None

    # ---------------------------------------------------------------- slicing
    def set_global_pop(self, n: int):
        self.global_pop = n

    def slice_of(self, n: int):
        return balanced_slices(n, self.world_size)[self.rank]

    # ---------------------------------------------------------------- collectives
    def all_gather_rows(self, local: torch.Tensor, n_total: Optional[int]) -> torch.Tensor:
        """Concatenate every rank's rows (rank order).  Uneven slices are padded to
        the largest slice for a single fixed-size collective, then compacted."""
        if self.world_size == 1:
            return local
        if n_total is None:
            sizes = torch.tensor([local.shape[0]], device=local.device)
            allsz = [torch.zeros_like(sizes) for _ in range(self.world_size)]
            dist.all_gather(allsz, sizes, group=self.group)
            counts = [int(s.item()) for s in allsz]
        else:
            counts = [s for _, s in balanced_slices(n_total, self.world_size)]
        mx = max(counts)
        local = local.contiguous()
        if local.shape[0] < mx:
            pad = torch.zeros((mx - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
            local = torch.cat([local, pad], 0)
        out = torch.empty((mx * self.world_size,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local, group=self.group)
        if all(c == mx for c in counts):
            return out
        return torch.cat([out[i * mx : i * mx + c] for i, c in enumerate(counts)], 0)

    def all_reduce_(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        if self.world_size > 1:
            dist.all_reduce(t, op=op, group=self.group)
        return t

    def all_reduce_min_loc(self, value: torch.Tensor, index: torch.Tensor):
        """Global (min value, index) as ONE collective: pack the order-preserving
        uint32 image of the f32 value with a 32-bit index into an int64 and reduce
        with MIN (SURVEY §2.11 "MINLOC")."""
        v = value.to(torch.float32).reshape(1)
        bits = v.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        neg = bits >= 0x80000000
        ordered = torch.where(neg, (~bits) & 0xFFFFFFFF, bits | 0x80000000)
        packed = (ordered << 31) | (index.to(torch.int64).reshape(1) & 0x7FFFFFFF)
        if self.world_size > 1:
            dist.all_reduce(packed, op=dist.ReduceOp.MIN, group=self.group)
        o = (packed >> 31) & 0xFFFFFFFF
        idx = packed & 0x7FFFFFFF
        neg = o < 0x80000000
        b = torch.where(neg, (~o) & 0xFFFFFFFF, o & 0x7FFFFFFF)
        b = torch.where(b >= 0x80000000, b - (1 << 32), b).to(torch.int32)
        return b.view(torch.float32).reshape(()), idx.reshape(())

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world_size > 1:
            dist.broadcast(t, src=src, group=self.group)
        return t

    def broadcast_state(self, state: State, src: int = 0) -> State:
        leaves, spec = tree_flatten(state)
        out = []
        for x in leaves:
            if isinstance(x, torch.Tensor):
                y = x.contiguous().clone()
                if y.dtype == torch.bool:
                    z = y.to(torch.uint8)
                    self.broadcast_(z, src)
                    y = z.to(torch.bool)
                else:
                    self.broadcast_(y, src)
                out.append(y)
            else:
                out.append(x)
        return tree_unflatten(out, spec)

    def barrier(self):
        if self.world_size > 1:
            dist.barrier(group=self.group)

    def state_checksum(self, state: State) -> torch.Tensor:
        """Cheap divergence detector: sum of every float leaf."""
        acc = None
        for x in tree_flatten(state)[0]:
            if isinstance(x, torch.Tensor) and x.is_floating_point():
                s = x.double().sum().reshape(1)
                acc = s if acc is None else acc + s
        return acc if acc is not None else torch.zeros(1, dtype=torch.float64)

    def check_replicas(self, state: State, atol: float = 0.0) -> bool:
        c = self.state_checksum(state)
        if self.world_size == 1:
            return True
        if self.backend == "nccl":
            c = c.to(torch.device("cuda", torch.cuda.current_device()))
        mx, mn = c.clone(), c.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=self.group)
        dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=self.group)
        return bool((mx - mn).abs().item() <= atol)


class SimulatedDistContext(DistContext):
    """Rank ``rank`` of a ``world``-rank job, simulated in ONE process on one device: every
    collective is replaced by a local operation on a buffer of the size the real collective
    would produce (all-gathers tile the local rows ``world`` times, all-reduces touch the
    buffer in place, broadcasts and barriers are no-ops).  ``bench.py --simulate-rank``
    uses it to time one rank's share of an N-GPU step (its critical path without the wire
    time of the collectives) on the single GPU a builder has; the selection then sees the
    local rows replicated, so the numerics are rank 0's shape of work, not the real run's."""

    def __init__(self, rank: int, world: int, algorithm=None):  # noqa: D401 — no process group
        self.group = None
        self.rank = int(rank)
        self.world_size = int(world)
        self.backend = "simulated"
        self.algorithm_sharded = algorithm is not None and hasattr(algorithm, "ask_sharded") and hasattr(algorithm, "tell_sharded")
        self.global_pop = None
        from .wire import WireCounters, WireModel

        self.wire = WireModel()
        self.counters = WireCounters()

    @property
    def bytes_all_reduce(self):
        return self.counters.all_reduce_bytes

    @property
    def bytes_all_gather(self):
        return self.counters.all_gather_bytes

    def _target(self):
        """The counters a call records into: during a graph capture the captured step's own
        counters (those calls repeat on every replay without running Python again)."""
        c = self.counters
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            # the workflow opened this variant's counters (begin_capture) before capturing; a
            # capture it did not announce gets counters of its own
            if c.captured is None:
                c.begin_capture(None)
            return c.captured
        return c

    def _count(self, kind: str, nbytes: int):
        c = self._target()
        if kind == "all_reduce":
            c.all_reduce_calls += 1
            c.all_reduce_bytes += nbytes
            c.wire_us += self.wire.all_reduce_us(nbytes, self.world_size)
        else:
            c.all_gather_calls += 1
            c.all_gather_bytes += nbytes
            c.wire_us += self.wire.all_gather_us(nbytes, self.world_size)

    def count_peer_rows(self, rows: torch.Tensor, row_bytes: int):
        """A peer row gather of ``rows`` (device scalar: rows that a real rank would read from
        other ranks' buffers) — accumulated on the device, read once after timing."""
        self._target().peer_gathers += 1
        c = self.counters  # the row count itself accumulates on the device, replays included
        c.row_bytes = int(row_bytes)
        r = rows.to(torch.float64).reshape(())
        if c.peer_rows is None:
            c.peer_rows = torch.zeros((), dtype=torch.float64, device=r.device)
        c.peer_rows.add_(r)

    def all_gather_rows(self, local: torch.Tensor, n_total: Optional[int]) -> torch.Tensor:
        counts = [s for _, s in balanced_slices(n_total, self.world_size)] if n_total is not None else [local.shape[0]] * self.world_size
        mx = max(counts)
        local = local.contiguous()
        if local.shape[0] < mx:
            pad = torch.zeros((mx - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
            local = torch.cat([local, pad], 0)
        out = local.repeat((self.world_size,) + (1,) * (local.dim() - 1))
        self._count("all_gather", out.numel() * out.element_size())
        if all(c == mx for c in counts):
            return out
        return torch.cat([out[i * mx : i * mx + c] for i, c in enumerate(counts)], 0)

    def all_reduce_(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        self._count("all_reduce", t.numel() * t.element_size())
        return t.mul_(1) if t.is_floating_point() else t

    def all_reduce_min_loc(self, value: torch.Tensor, index: torch.Tensor):
        self._count("all_reduce", 8)  # one packed u64 MINLOC
        return value.reshape(()), index.reshape(())

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        return t

    def barrier(self):
        return None
