"""Workflow marker class (reference ``src/evox/core/workflow.py:4-5``)."""
from .module import Stateful


class Workflow(Stateful):
    pass
