from . import de_variants
from .de_variants import *  # noqa
from .pso_variants import *  # noqa
from .es_variants import *  # noqa
