from .nsga2 import NSGA2
from .moead import MOEAD
