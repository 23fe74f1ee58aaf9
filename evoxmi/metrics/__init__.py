"""Multi-objective quality indicators (reference ``src/evox/metrics``): GD, GD+, IGD,
IGD+, and the hypervolume (Monte-Carlo estimators of the reference plus exact
2-/3-objective hypervolume)."""
from .gd import GD, GDPlus, gd, gd_plus
from .igd import IGD, IGDPlus, igd, igd_plus
from .hypervolume import HV, bounding_cube_monte_carlo_hv, each_cube_monte_carlo_hv, exact_hv

__all__ = ["GD", "GDPlus", "IGD", "IGDPlus", "HV", "gd", "gd_plus", "igd", "igd_plus", "exact_hv",
           "bounding_cube_monte_carlo_hv", "each_cube_monte_carlo_hv"]
