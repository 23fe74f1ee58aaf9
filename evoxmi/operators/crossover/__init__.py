from .differential_evolution import (
    DifferentialEvolve, batched_de_arith_recom, batched_de_bin_cross, batched_de_diff_sum, batched_de_diff_sum_archive,
    batched_de_diff_sum_rank, batched_de_exp_cross, de_arith_recom, de_bin_cross, de_diff_sum, de_diff_sum_archive,
    de_diff_sum_rank, de_exp_cross, differential_evolve, move_n_small_numbers,
)
from .sbx import OnePoint, SBXCrossover, SimulatedBinary, UniformRand, one_point, sbx, simulated_binary, uniform_crossover
