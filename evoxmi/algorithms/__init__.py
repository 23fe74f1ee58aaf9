from .so import *  # noqa
from .mo import *  # noqa
