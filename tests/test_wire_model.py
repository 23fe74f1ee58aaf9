"""xGMI wire model and the simulated context's counters (evoxmi/parallel/wire.py)."""
import pytest
import torch

from evoxmi.parallel.wire import WireCounters, WireModel


def test_wire_model_formulas():
    m = WireModel(link_gbps=64, latency_us=10, peer_latency_us=2)
    assert m.all_reduce_us(1e6, 1) == 0.0
    assert m.all_reduce_us(64e3, 8) == pytest.approx(2 * 7 / 8 * 1.0 + 10)
    assert m.all_gather_us(8 * 64e3, 8) == pytest.approx(1.0 + 10)
    assert m.peer_read_us(7 * 64e3, 8) == pytest.approx(1.0 + 2)
    assert m.peer_read_us(0, 8) == 0.0


def test_eager_summary_counts_every_generation():
    m = WireModel()
    c = WireCounters()
    for _ in range(4):
        c.all_reduce_calls += 1
        c.all_reduce_bytes += 800
        c.wire_us += m.all_reduce_us(800, 8)
    c.peer_gathers = 4
    c.row_bytes = 4000
    c.peer_rows = torch.tensor(400.0, dtype=torch.float64)
    s = c.summary(4, m, 8)
    assert s["all_reduce_per_gen"] == 1.0
    assert s["peer_bytes_per_gen"] == 100 * 4000
    assert s["wire_bytes_per_gen"] == pytest.approx(800 * 2 * 7 / 8 + 100 * 4000)


def test_graph_summary_uses_the_captured_step_and_averages_device_rows():
    """Graph replays: the host counters of the captured step stand for every generation, the
    device peer-row count accumulated over all replays is averaged; reset keeps row_bytes."""
    m = WireModel()
    c = WireCounters()
    c.row_bytes = 4000
    c.peer_rows = torch.tensor(0.0, dtype=torch.float64)
    cap = WireCounters(all_reduce_calls=2, all_reduce_bytes=1600, peer_gathers=1)
    cap.wire_us = 2 * m.all_reduce_us(800, 8)
    c.captured = cap
    c.reset()
    assert c.row_bytes == 4000 and c.captured is cap
    c.peer_rows += 5 * 120  # five replays, 120 rows each
    s = c.summary(5, m, 8, graph=True)
    assert s["all_reduce_per_gen"] == 2.0
    assert s["peer_bytes_per_gen"] == pytest.approx(120 * 4000)
    assert s["wire_ms_per_gen"] == pytest.approx((cap.wire_us + m.peer_read_us(120 * 4000, 8)) / 1e3)
    assert cap.peer_rows is None  # the captured counters are not mutated


def test_graph_summary_weights_every_captured_variant_by_its_replays():
    """Per-variant captured counters (CMA-ES replays a cold, an 8-slot and a late graph): the
    graph summary is Σ_v replays_v × counters_v per replayed generation, and a segmented capture's
    segments all add into their variant's counters."""
    from evoxmi.parallel.wire import WireCounters, WireModel

    c = WireCounters()
    a = c.begin_capture("cold")
    a.all_reduce_calls, a.all_reduce_bytes, a.wire_us = 2, 4000, 20.0
    a.all_reduce_calls += 1  # a second segment of the same capture
    a.all_reduce_bytes += 1000
    b = c.begin_capture("late")
    b.all_gather_calls, b.all_gather_bytes, b.wire_us = 1, 8000, 10.0
    for _ in range(3):
        c.note_replay("cold")
    c.note_replay("late")
    s = c.summary(4, WireModel(), 8, graph=True)
    assert s["all_reduce_per_gen"] == 3 * 3 / 4 and s["all_gather_per_gen"] == 1 / 4
    assert abs(s["wire_ms_per_gen"] - (3 * 20.0 + 10.0) / 4 / 1e3) < 1e-12
    c.reset()  # timed window: replay counts restart, the captured counters stay
    assert c.replays == {} and set(c.captured_by) == {"cold", "late"}
    c.note_replay("late")
    assert c.summary(1, WireModel(), 8, graph=True)["all_gather_per_gen"] == 1
