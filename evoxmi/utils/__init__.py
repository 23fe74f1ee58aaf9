from .common import *  # noqa: F401,F403
from .common import (
    AggregationFunction,
    TreeAndVector,
    compose,
    dominate_relation,
    min_by,
    parse_opt_direction,
    rank,
    rank_based_fitness,
    to_x32_if_needed,
    x32_func_call,
)
from .optim import OptaxWrapper, OptimizerWrapper, adam, clipup, get_optimizer, sgd
from .profiling import PhaseTimer, trace_range
