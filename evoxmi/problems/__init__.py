from . import numerical
from . import neuroevolution
from . import evoxbench
