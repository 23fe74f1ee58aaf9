import torch, sys
torch.set_printoptions(precision=3, linewidth=200, threshold=100000)
from evoxmi import config
from evoxmi import random as rnd
from evoxmi.algorithms import CMAES
from evoxmi.ops import sbr_device
from evoxmi.problems.numerical import CEC2022TestSuit
from evoxmi.workflows import StdWorkflow
for seed in (1, 2):
    center = (torch.rand(1000, generator=torch.Generator().manual_seed(seed)) * 160 - 80).cuda()
    algo = CMAES(center_init=center, init_stdev=20.0)
    wf = StdWorkflow(algo, CEC2022TestSuit.create(1), graph=False)
    st = wf.init(rnd.PRNGKey(2024, device=torch.device("cuda")))
    snap = sbr_device.snapshot_counts()
    for _ in range(200):
        st = wf.step(st)
    torch.cuda.synchronize()
    h = sbr_device.histories_since(snap)
    print("seed", seed, "deep iters", sbr_device.schedule("deep", 1000).iters)
    print(h, flush=True)
