"""Execution runtime helpers (hipGraph segments with host phases)."""
from .graph import SegmentedGraph, capturing, host_phase

__all__ = ["SegmentedGraph", "capturing", "host_phase"]
