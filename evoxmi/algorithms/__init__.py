from .so import *  # noqa
