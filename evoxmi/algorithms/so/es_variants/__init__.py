"""Evolution strategies (reference ``algorithms/so/es_variants/``)."""
from .cma_es import CMAES, SepCMAES, IPOPCMAES, BIPOPCMAES
from .ma_es import MAES, LMMAES
from .rmes import RMES
from .amalgam import AMaLGaM, IndependentAMaLGaM
from .nes import XNES, SeparableNES
from .open_es import OpenES
from .pgpe import PGPE, ClipUp
from .snes import SNES
from .des import DES
from .ars import ARS
from .esmc import ESMC
from .guided_es import GuidedES
from .asebo import ASEBO
from .cr_fm_nes import CR_FM_NES
from .persistent_es import PersistentES
from .noise_reuse_es import NoiseReuseES, Noise_reuse_es
from .les import LES
from ._common import sort_by_key
