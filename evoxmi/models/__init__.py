"""Policy / model definitions for neuroevolution (the reference uses flax modules)."""
from .mlp import MLPPolicy

__all__ = ["MLPPolicy"]
