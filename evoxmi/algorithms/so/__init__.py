from .pso_variants import *  # noqa
from .es_variants import *  # noqa
