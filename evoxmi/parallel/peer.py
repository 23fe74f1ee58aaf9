"""Direct peer buffers over xGMI: every rank exposes one device buffer that the other ranks
of the node read with ordinary loads (IPC-mapped, ``hipIpcGetMemHandle`` / ``OpenMemHandle``).

RCCL's collectives move whole tensors; some exchanges need only a data-dependent subset of
rows from each peer — MOEA/D's owner-computes tell pulls the winning offspring rows of the
slots a rank keeps current (``algorithms/mo/moead.py``).  A gather kernel that reads those
rows straight out of the generating rank's memory is the "direct mesh" path of SURVEY
§2.3: every GPU reads its rows from all 7 peers concurrently, one link per peer, with no
host involvement (capturable, sizes decided on the device).  Handles are exchanged once
through ``torch.distributed`` (``all_gather_object``).

Memory model (round 6: explicit, not left to cache side effects).  Peer buffers are plain
``hipMalloc`` allocations (coarse-grained): peers read them over xGMI, and those reads are
served from the owner's HBM through its memory-side cache, NOT from the owner's L2 — nor
is a reader's L2 kept coherent with another GPU's writes.  So every exchange is:

1. writer: the kernels that fill the owner's buffer, then :meth:`PeerBuffer.release` — a
   one-thread kernel with a system-scope release fence (``peer_release``: the owner's dirty L2
   lines are written back to HBM) — all on the owner's stream;
2. a collective between writer and reader (the fitness all-gather / z_max all-reduce of the
   same generation): RCCL orders the reader's later kernels after the owner's earlier ones;
3. reader: a system-scope acquire launch right before the gather kernel (``moead_halo_gather``:
   lines of the peer buffer left in any XCD's caches by the previous generation's reads are
   invalidated), then the gather reads the rows non-temporally (read once);
4. reuse: the owner must not rewrite the buffer before every reader is done — the owner calls
   :meth:`PeerBuffer.fence` (a one-float all-reduce) after its reads.

Each fence is one lane of 64 workgroups (a fence acts on its CU's L1 and its XCD's L2; blocks are
dealt round-robin over the 8 XCDs): one launch per generation on each side (cost measured in
profiles/NOTES.md, round 6 — a fence in every reading wave instead cost 0.21 ms per generation).  Backends without device IPC (CPU / gloo on
CPU tensors) fall back to an all-gather of the full buffers (``peer_table`` returns
``None``); the single-process :class:`SimulatedDistContext` points every peer entry at the
local buffer (same rows read from local HBM).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import _ext


class PeerBuffer:
    def __init__(self, ctx, rows: int, cols: int, device):
        self.ctx = ctx
        self.rows, self.cols = rows, cols
        self.device = torch.device(device)
        self.ipc = self.device.type == "cuda" and ctx.world_size > 1 and getattr(ctx, "backend", "") != "simulated"
        self._opened = []
        if self.ipc:
            self.local = _ext.ops().ipc_alloc(rows * cols, self.device.index or 0).view(rows, cols)
            ok, ptrs = True, []
            try:
                h = _ext.ops().ipc_handle(self.local)
            except RuntimeError:
                h, ok = None, False
            handles = [None] * ctx.world_size
            dist.all_gather_object(handles, h, group=ctx.group)
            ok = ok and all(x is not None for x in handles)
            for r, hr in enumerate(handles if ok else []):
                if r == ctx.rank:
                    ptrs.append(self.local.data_ptr())
                    continue
                try:
                    p = _ext.ops().ipc_open(hr, self.device.index or 0)
                except RuntimeError:
                    ok = False
                    break
                self._opened.append(p)
                ptrs.append(p)
            # every rank must agree on the path (a rank that cannot map a peer → all fall back)
            flag = [None] * ctx.world_size
            dist.all_gather_object(flag, ok, group=ctx.group)
            self.ipc = all(flag)
            if not self.ipc:
                self.close()
            self.table = torch.tensor(ptrs, dtype=torch.int64, device=self.device) if self.ipc else None
        elif self.device.type == "cuda" and getattr(ctx, "backend", "") == "simulated":
            # one rank's share of an N-GPU step in one process: every "peer" buffer is this
            # rank's own, so the gather reads the same rows from local HBM instead of xGMI
            self.local = torch.zeros(rows, cols, device=self.device)
            self.table = torch.full((ctx.world_size,), self.local.data_ptr(), dtype=torch.int64, device=self.device)
        else:
            self.local = torch.zeros(rows, cols, device=self.device)
            self.table = None
        self._one = torch.zeros(1, device=self.device)

    def peer_table(self):
        """int64 device pointers of every rank's buffer (None: no device IPC)."""
        return self.table

    def release(self):
        """Writer side of the contract: system-scope release after this rank filled ``local``
        (a no-op without device IPC — the all-gather fallback and the simulated rank read
        through the normal stream order — except that the simulated rank runs the kernel, so
        its cost is in the one-GPU projection)."""
        if self.device.type == "cuda" and (self.ipc or getattr(self.ctx, "backend", "") == "simulated"):
            _ext.ops().peer_release(self.device.index or 0)

    def fence(self):
        """All ranks have finished reading every peer buffer (before the owners rewrite them)."""
        if self.ipc:
            self.ctx.all_reduce_(self._one)
        elif getattr(self.ctx, "backend", "") == "simulated":
            self.ctx._count("all_reduce", 4)  # the real run's one-float fence (wire accounting)

    def close(self):
        for p in self._opened:
            _ext.ops().ipc_close(p)
        self._opened = []
