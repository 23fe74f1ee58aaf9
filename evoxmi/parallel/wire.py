"""xGMI wire-time model for one rank's share of an N-GPU step (the single-GPU simulation of
``SimulatedDistContext`` replaces every collective and peer read by a local operation, so
its measured time leaves the wire out).

MI355X node topology: 8 GPUs fully connected by point-to-point xGMI links,
7 per GPU.  The model is deliberately conservative and states its constants:

* all-reduce of S bytes: ring, bound by one link per hop — 2(N−1)/N · S / B_link, plus one
  collective latency α;
* all-gather of a T-byte result from N equal shards: direct (mesh) — every rank receives its
  N−1 peers' shards on N−1 links concurrently — (T/N) / B_link + α;
* peer (IPC) row reads of R bytes spread over the peers (MOEA/D halo gather): R / ((N−1)·B_link)
  plus a per-gather latency α_peer.

Defaults: B_link = 64 GB/s per link per direction (a sustained fraction of the link's
peak), α = 10 µs per RCCL collective, α_peer = 2 µs.  Projections add the wire time to the
measured compute time (no overlap credited).
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Dict


@dataclass
class WireModel:
    link_gbps: float = 64.0
    latency_us: float = 10.0
    peer_latency_us: float = 2.0

    def _bps(self) -> float:
        return self.link_gbps * 1e9

    def all_reduce_us(self, nbytes: float, world: int) -> float:
        if world <= 1:
            return 0.0
        return 2.0 * (world - 1) / world * nbytes / self._bps() * 1e6 + self.latency_us

    def all_gather_us(self, total_bytes: float, world: int) -> float:
        if world <= 1:
            return 0.0
        return total_bytes / world / self._bps() * 1e6 + self.latency_us

    def peer_read_us(self, nbytes: float, world: int) -> float:
        if world <= 1 or nbytes <= 0:
            return 0.0
        return nbytes / ((world - 1) * self._bps()) * 1e6 + self.peer_latency_us

    def describe(self) -> Dict[str, float]:
        return {"link_GBps_per_direction": self.link_gbps, "collective_latency_us": self.latency_us,
                "peer_gather_latency_us": self.peer_latency_us}


@dataclass
class WireCounters:
    """Per-rank communication volume accumulated by a (simulated) context."""

    all_reduce_calls: int = 0
    all_reduce_bytes: int = 0           # payload per rank (the reduced tensor's size)
    all_gather_calls: int = 0
    all_gather_bytes: int = 0           # size of the gathered result
    peer_gathers: int = 0
    peer_rows: object = None            # device scalar: rows read from other ranks (no host sync)
    row_bytes: int = 0
    wire_us: float = 0.0                # modelled wire time of the recorded collectives
    per_call: Dict[str, int] = field(default_factory=dict)

    captured: object = None              # counters of the most recently captured step
    # per graph variant (Algorithm.graph_variant): the captured step's counters (every segment of a
    # segmented capture adds into its variant's), and how many replays of it the counters cover
    captured_by: Dict[object, "WireCounters"] = field(default_factory=dict)
    replays: Dict[object, int] = field(default_factory=dict)

    def reset(self):
        """Zero the host counters, the replay counts and the device peer-row count (in place: a
        captured graph keeps accumulating into the same tensor on every replay); the captured
        steps' counters stay (the graphs are not re-captured)."""
        pr, cap, rb, by = self.peer_rows, self.captured, self.row_bytes, self.captured_by
        self.__init__()
        if pr is not None:
            pr.zero_()
            self.peer_rows = pr
        self.captured = cap
        self.captured_by = by
        self.row_bytes = rb  # a property of the problem (bytes of one decision row), not a count

    def begin_capture(self, key) -> "WireCounters":
        """Fresh counters for the capture of graph variant ``key`` (its segments all add into them)."""
        c = self.captured_by[key] = WireCounters()
        self.captured = c
        return c

    def note_replay(self, key) -> None:
        self.replays[key] = self.replays.get(key, 0) + 1

    def _replayed_total(self) -> "WireCounters":
        """The host counters of every replay: each variant's captured step × its replay count."""
        t = WireCounters()
        for key, n in self.replays.items():
            c = self.captured_by.get(key)
            if c is None:
                continue
            t.all_reduce_calls += n * c.all_reduce_calls
            t.all_reduce_bytes += n * c.all_reduce_bytes
            t.all_gather_calls += n * c.all_gather_calls
            t.all_gather_bytes += n * c.all_gather_bytes
            t.peer_gathers += n * c.peer_gathers
            t.wire_us += n * c.wire_us
            t.row_bytes = t.row_bytes or c.row_bytes
        return t

    def summary(self, steps: int, model: WireModel, world: int, graph: bool = False) -> Dict[str, float]:
        """Per-generation volumes over ``steps`` generations.  ``graph``: the generations were
        hipGraph replays, whose host-side collective calls ran once, at capture — the host
        counters of that captured step stand for every replay; the device peer-row count
        accumulated on every replay."""
        steps = max(1, int(steps))
        if graph and self.replays and self.captured_by:
            # replays of several variants (e.g. CMA-ES's cold / 8-slot / late eigensolver
            # schedules), each weighted by how many generations replayed it
            t = self._replayed_total()
            t.peer_rows = 0.0 if self.peer_rows is None else float(self.peer_rows)
            t.row_bytes = self.row_bytes or t.row_bytes
            return WireCounters.summary(t, sum(self.replays.values()), model, world)
        if graph and self.captured is not None:
            # one generation = the captured step's host counters, with the device peer-row count
            # (accumulated over `steps` replays) averaged to one generation
            rows = 0.0 if self.peer_rows is None else float(self.peer_rows) / steps
            c = replace(self.captured, peer_rows=rows, row_bytes=self.row_bytes or self.captured.row_bytes, captured=None)
            return WireCounters.summary(c, 1, model, world)
        peer_rows = 0.0 if self.peer_rows is None else float(self.peer_rows)  # tensor or float
        peer_bytes = peer_rows * self.row_bytes
        peer_us = sum(model.peer_read_us(peer_bytes / max(1, self.peer_gathers), world) for _ in range(self.peer_gathers)) \
            if self.peer_gathers else 0.0
        return {
            "all_reduce_per_gen": self.all_reduce_calls / steps,
            "all_gather_per_gen": self.all_gather_calls / steps,
            "collective_bytes_per_gen": (self.all_reduce_bytes + self.all_gather_bytes // max(1, world)) / steps,
            "peer_bytes_per_gen": peer_bytes / steps,
            "wire_bytes_per_gen": (self.all_reduce_bytes * 2 * (world - 1) / world + self.all_gather_bytes * (world - 1) / world
                                   + peer_bytes) / steps,
            "wire_ms_per_gen": (self.wire_us + peer_us) / steps / 1e3,
        }
