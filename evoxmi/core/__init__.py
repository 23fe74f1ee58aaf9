from .state import State, tree_map, tree_leaves, tree_flatten, tree_unflatten, tree_structure
from .module import (
    Stateful,
    StackedModules,
    use_state,
    jit_method,
    jit_class,
    dataclass,
    Static,
    Stack,
    stack_states,
)
from .algorithm import Algorithm, algorithm_has_init_ask
from .problem import Problem
from .monitor import Monitor
from .workflow import Workflow, capture_warmup, in_capture_warmup
from .checkpoint import save_state, load_state
