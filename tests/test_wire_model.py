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
