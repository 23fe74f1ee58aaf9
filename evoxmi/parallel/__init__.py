"""Distributed execution (SPMD, one process per GPU, RCCL over xGMI)."""
from .bootstrap import init_distributed, destroy, env_world
from .context import DistContext, balanced_slices
