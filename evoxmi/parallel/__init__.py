"""Distributed execution (SPMD, one process per GPU, RCCL over xGMI)."""
from .bootstrap import init_distributed, destroy, env_world
from .context import DistContext, balanced_slices
from .dim_sharded import DimShardedProblem, dim_sharded_fitness, supports_dim_sharding
from .resilience import FaultInjector, Heartbeat, InjectedFault, latest_checkpoint, run_elastic
