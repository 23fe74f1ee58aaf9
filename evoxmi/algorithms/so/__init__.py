from .pso_variants import *  # noqa
