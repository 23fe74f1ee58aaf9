from .non_dominate import (
    NonDominate, crowding_distance, crowding_distance_sort, lexsort, non_dominate, non_dominated_sort,
    host_rank_from_domination_matrix,
)
from .misc import (
    ReferenceVectorGuided, RouletteWheelSelection, TopkFit, Tournament, UniformRand, move_n_small_numbers,
    ref_vec_guided, select_rand_pbest, topk_fit, tournament_multi_fit, tournament_single_fit, uniform_rand,
)
