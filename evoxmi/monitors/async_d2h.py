"""Asynchronous device→host transfer for monitors (the reference's
``io_callback`` host callbacks become stream-ordered copies that never stall compute).

:class:`D2HCopier` snapshots a device tensor on the compute stream (a device-to-device
clone: the source may be a graph's static buffer that the next replay overwrites), then
copies the snapshot into pinned host memory on a dedicated copy stream, so the DMA
overlaps the following generations.  :class:`HostList` holds the pending copies and
resolves an entry (waits for its copy event only) when it is read.
"""
from __future__ import annotations

import torch


class PendingHost:
    __slots__ = ("host", "group")

    def __init__(self, host: torch.Tensor, group):
        self.host, self.group = host, group

    def get(self) -> torch.Tensor:
        if self.group is not None:
            self.group.wait()
            self.group = None
        return self.host


def _resolve(x):
    return x.get() if isinstance(x, PendingHost) else x


class HostList(list):
    """A list whose PendingHost entries resolve to their host tensors on access."""

    def __getitem__(self, i):
        v = super().__getitem__(i)
        return [_resolve(x) for x in v] if isinstance(i, slice) else _resolve(v)

    def __iter__(self):
        for v in super().__iter__():
            yield _resolve(v)


class _Group:
    """Snapshots staged back to back in one device chunk, moved to one pinned host chunk by a
    single side-stream copy."""

    def __init__(self, dev, nbytes, host_buf):
        self.dev_buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self.host_buf = host_buf
        self.used = 0
        self.count = 0
        self.event = None
        self.copier = None

    def carve(self, buf, off, shape, dtype):
        n = int(torch.Size(shape).numel())
        return buf[off:].view(dtype)[:n].view(shape)

    def wait(self):
        if self.event is None:  # not yet flushed: issue the copy now
            self.copier._flush(self)
        self.event.synchronize()


class D2HCopier:
    """Device→host history copies that never stall the generation loop.

    A snapshot is one device-to-device copy on the compute stream into a staging chunk (the
    source may be a graph's static buffer that the next replay overwrites); every
    ``flush_every`` snapshots (or when the chunk is full, or when an entry is read) the chunk
    goes to pinned host memory with ONE copy on a dedicated stream.  A side-stream copy plus
    event per generation measured +0.39 ms per CMA-ES generation on the flagship; staged it
    costs what a device-kept history does (profiles/r3_bench_monitor_modes.txt)."""

    MIN_CHUNK_BYTES = 64 << 10

    ARENA_BYTES = 32 << 20

    def __init__(self, flush_every: int = 16, side_stream: bool = None):
        import os

        # the chunk copy is enqueued on the compute stream by default: one ordered async DMA per
        # flush_every generations; a separate copy stream (wait_stream + event per flush) cost
        # the hipGraph-replayed flagship ≈4 ms per flush on the box
        self.side_stream = bool(int(os.environ.get("EVOXMI_D2H_SIDE_STREAM", "0"))) if side_stream is None else side_stream
        self._streams = {}
        self._groups = {}
        self.flush_every = flush_every
        self._arena = None
        self._arena_off = 0

    def _host_chunk(self, nbytes):
        """Pinned host memory for one group, carved from large arenas (a page-locking
        allocation per group cost ≈3 ms each on the box)."""
        if self._arena is None or self._arena_off + nbytes > self._arena.numel():
            self._arena = torch.empty(max(self.ARENA_BYTES, nbytes), dtype=torch.uint8, pin_memory=True)
            self._arena_off = 0
        v = self._arena[self._arena_off : self._arena_off + nbytes]
        self._arena_off += nbytes
        return v

    def _stream(self, dev: torch.device) -> torch.cuda.Stream:
        if dev not in self._streams:
            self._streams[dev] = torch.cuda.Stream(device=dev)
        return self._streams[dev]

    def _flush(self, g: _Group):
        dev = g.dev_buf.device
        if self._groups.get(dev) is g:
            del self._groups[dev]
        if self.side_stream:
            s = self._stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
        else:
            s = torch.cuda.current_stream(dev)
        with torch.cuda.stream(s):
            g.host_buf[: g.used].copy_(g.dev_buf[: g.used], non_blocking=True)
            g.event = torch.cuda.Event()
            g.event.record(s)
        if self.side_stream:
            g.dev_buf.record_stream(s)
        # release the staging chunk now: the caching allocator orders its reuse after the copy
        # already enqueued on the compute stream (record_stream covers the side-stream case), so
        # a history read only at the end of a run does not keep every snapshot on the device too
        g.dev_buf = None

    def submit(self, x: torch.Tensor):
        if not x.is_cuda:
            return x.detach().clone()
        if torch.cuda.is_current_stream_capturing():
            # inside a graph capture: a host copy cannot be captured; keep a device snapshot
            return x.detach().clone()
        dev = x.device
        nbytes = (max(1, x.numel() * x.element_size()) + 255) & ~255
        g = self._groups.get(dev)
        if g is not None and g.used + nbytes > g.dev_buf.numel():
            self._flush(g)
            g = None
        if g is None:
            size = max(self.MIN_CHUNK_BYTES, nbytes * self.flush_every)
            g = self._groups[dev] = _Group(dev, size, self._host_chunk(size))
            g.copier = self
        g.carve(g.dev_buf, g.used, x.shape, x.dtype).copy_(x.detach())
        host = g.carve(g.host_buf, g.used, x.shape, x.dtype)
        g.used += nbytes
        g.count += 1
        if g.count >= self.flush_every:
            self._flush(g)
        return PendingHost(host, g)

    def flush(self):
        for g in list(self._groups.values()):
            self._flush(g)
