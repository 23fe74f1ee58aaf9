from .eval_monitor import EvalMonitor
from .pop_monitor import PopMonitor
from .std_so_monitor import StdSOMonitor
from .std_mo_monitor import StdMOMonitor
from .evoxvis_monitor import EvoXVisMonitor, read_evoxvis
from .throughput_monitor import ThroughputMonitor, JSONLLogger
