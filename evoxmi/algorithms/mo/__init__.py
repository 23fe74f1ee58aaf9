"""Multi-objective algorithms (reference ``algorithms/mo/``)."""
from .nsga2 import NSGA2
from .nsga3 import NSGA3
from .moead import MOEAD
from .moeaddra import MOEADDRA
from .moeadm2m import MOEADM2M
from .eagmoead import EAGMOEAD
from .rvea import RVEA
from .rveaa import RVEAa
from .ibea import IBEA
from .bce_ibea import BCEIBEA
from .hype import HypE
from .spea2 import SPEA2
from .gde3 import GDE3
from .knea import KnEA
from .bige import BiGE
from .sra import SRA
from .tdea import TDEA
from .lmocso import LMOCSO
from .im_moea import IMMOEA

__all__ = ["NSGA2", "NSGA3", "MOEAD", "MOEADDRA", "MOEADM2M", "EAGMOEAD", "RVEA", "RVEAa", "IBEA", "BCEIBEA", "HypE", "SPEA2",
           "GDE3", "KnEA", "BiGE", "SRA", "TDEA", "LMOCSO", "IMMOEA"]
