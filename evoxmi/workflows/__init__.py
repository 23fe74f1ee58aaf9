from .std_workflow import StdWorkflow
from .non_jit_workflow import NonJitWorkflow
from .distributed import RayDistributedWorkflow, ShardedWorkflow
