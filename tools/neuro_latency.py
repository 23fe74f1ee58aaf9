import sys, time, torch
sys.path.insert(0, "/root/repo")
from evoxmi import random as rnd
from evoxmi.ops import neuro
from evoxmi.problems.neuroevolution.reinforcement_learning.envs import get_environment
h = 64
P = neuro.ant_param_count(h, h)
s0, _ = get_environment("ant").reset(rnd.PRNGKey(0), 1)
init = s0[0].cuda()
pops = [int(a) for a in sys.argv[1:]] or [64, 8192]
for pop in pops:
    W = torch.zeros(pop, P, device="cuda")
    for cap in (0, 1, 10, 50, 200, 1000):
        neuro.ant_rollout(W, h, h, init, cap); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            neuro.ant_rollout(W, h, h, init, cap)
        e1.record(); torch.cuda.synchronize()
        print(pop, cap, round(e0.elapsed_time(e1) / 3, 3), "ms", flush=True)
