from . import crossover, mutation, sampling, selection
from .crossover import *  # noqa
from .mutation import Bitflip, Gaussian, Polynomial, bitflip, gaussian, polynomial
from .sampling import GridSampling, LatinHypercubeSampling, UniformSampling
from .selection import *  # noqa
