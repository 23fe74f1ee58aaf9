"""Visualisation helpers (reference ``src/evox/vis_tools``)."""
from . import plot
