"""Differential-evolution zoo (reference ``algorithms/so/de_variants/``)."""
from .de import DE
from .ode import ODE
from .code import CoDE
from .jade import JaDE
from .sade import SaDE
from .shade import SHADE
from .lshade import LSHADE, ILSHADE, JSO, LSHADE_RSP
from .epsde import EPSDE
from .evde import EVDE

__all__ = ["DE", "ODE", "CoDE", "JaDE", "SaDE", "SHADE", "LSHADE", "ILSHADE", "JSO", "LSHADE_RSP", "EPSDE", "EVDE"]
