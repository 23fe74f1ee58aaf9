"""evoxmi — an MI355X-native evolutionary-computation framework.

Programming model (parity with EvoX / MinyangChen/evox-myc): ``Stateful`` modules
with immutable hierarchical ``State``, ``Algorithm.ask/tell``,
``Problem.evaluate``, monitors hooked into a ``StdWorkflow`` that runs one
generation per ``step``.  Execution model: PyTorch-ROCm tensors in HBM,
hand-written HIP kernels for the population hot path (``evoxmi/_C.so``, built
for gfx950), hipGraph-captured generations and RCCL collectives for
one-process-per-GPU SPMD runs.
"""
from .core import (
    Algorithm,
    Monitor,
    Problem,
    Stack,
    State,
    Stateful,
    StackedModules,
    Static,
    Workflow,
    dataclass,
    jit_class,
    jit_method,
    use_state,
)
from .ops import random
from . import utils

__version__ = "0.1.0"


def __getattr__(name):
    # lazy sub-packages keep `import evoxmi` cheap
    import importlib

    if name in ("algorithms", "problems", "workflows", "monitors", "operators", "metrics", "parallel", "models", "vis_tools", "ops"):
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
