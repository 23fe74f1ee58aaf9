"""Multi-process workflows.

* :class:`ShardedWorkflow` — the MI355X-native SPMD workflow: one process per GPU
  (launched by ``torchrun``), RCCL collectives, replicated optimiser state,
  population-sharded generation/evaluation (SURVEY §7.1 "Distributed").
* :class:`RayDistributedWorkflow` — API-compatible replacement for the reference's
  Ray actor workflow (``src/evox/workflows/distributed.py:229-361``); see
  :mod:`evoxmi.workflows.process_workflow`.
"""
from __future__ import annotations

from ..parallel.bootstrap import init_distributed
from .std_workflow import StdWorkflow


class ShardedWorkflow(StdWorkflow):
    """``StdWorkflow`` that joins the default process group and shards itself on ``init``."""

    def init(self, key=None, no_state: bool = False):
        init_distributed()
        state = super().init(key, no_state)
        return self.enable_distributed(state)


from .process_workflow import RayDistributedWorkflow  # noqa: E402
