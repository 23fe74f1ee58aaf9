"""Particle-swarm zoo (reference ``algorithms/so/pso_variants/``)."""
from .pso import PSO
from .cso import CSO
from .clpso import CLPSO
from .sl_pso import SLPSOGS, SLPSOUS
from .dms_pso_el import DMSPSOEL
from .fips import FIPS
from .swmmpso import SwmmPSO
from .fs_pso import FSPSO
from . import topology_utils
