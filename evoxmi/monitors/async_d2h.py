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
    __slots__ = ("host", "event")

    def __init__(self, host: torch.Tensor, event):
        self.host, self.event = host, event

    def get(self) -> torch.Tensor:
        if self.event is not None:
            self.event.synchronize()
            self.event = None
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


class D2HCopier:
    def __init__(self):
        self._streams = {}

    def _stream(self, dev: torch.device) -> torch.cuda.Stream:
        if dev not in self._streams:
            self._streams[dev] = torch.cuda.Stream(device=dev)
        return self._streams[dev]

    def submit(self, x: torch.Tensor):
        if not x.is_cuda:
            return x.detach().clone()
        if torch.cuda.is_current_stream_capturing():
            # inside a graph capture: a host copy cannot be captured; keep a device snapshot
            return x.detach().clone()
        snap = x.detach().clone()  # on the compute stream, ordered after the producer
        s = self._stream(x.device)
        s.wait_stream(torch.cuda.current_stream(x.device))
        host = torch.empty(x.shape, dtype=x.dtype, pin_memory=True)
        with torch.cuda.stream(s):
            host.copy_(snap, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(s)
        snap.record_stream(s)  # the allocator keeps the snapshot alive until the copy ran
        return PendingHost(host, ev)
