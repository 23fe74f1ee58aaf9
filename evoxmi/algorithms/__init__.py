from .so import *  # noqa
from .mo import *  # noqa
from .containers import *  # noqa
from . import containers
