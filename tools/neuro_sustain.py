"""Per-call time of back-to-back fused Ant rollouts (pop 1024, zero weights, cap 1000): does
the per-step latency drift under sustained load?"""
import sys, time, torch
sys.path.insert(0, "/root/repo")
from evoxmi import random as rnd
from evoxmi.ops import neuro
from evoxmi.problems.neuroevolution.reinforcement_learning.envs import get_environment

h, pop, n = 64, int(sys.argv[1]) if len(sys.argv) > 1 else 1024, int(sys.argv[2]) if len(sys.argv) > 2 else 200
P = neuro.ant_param_count(h, h)
s0, _ = get_environment("ant").reset(rnd.PRNGKey(0), 1)
init = s0[0].cuda()
mode = sys.argv[3] if len(sys.argv) > 3 else "zeros"
if mode == "zeros":
    W = torch.zeros(pop, P, device="cuda")
elif mode == "negzero":
    W = torch.full((pop, P), -0.0, device="cuda")
else:  # 0 · randn: signed zeros in a random pattern
    W = 0.0 * torch.randn(pop, P, device="cuda", generator=torch.Generator(device="cuda").manual_seed(0))
ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
neuro.ant_rollout(W, h, h, init, 1000)
torch.cuda.synchronize()
ev[0].record()
for i in range(n):
    neuro.ant_rollout(W, h, h, init, 1000)
    ev[i + 1].record()
torch.cuda.synchronize()
ts = [ev[i].elapsed_time(ev[i + 1]) for i in range(n)]
print(mode, "mean", round(sum(ts) / n, 3))
print("first5", [round(t, 2) for t in ts[:5]], "last5", [round(t, 2) for t in ts[-5:]])
# idle gap then again
time.sleep(2.0)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); neuro.ant_rollout(W, h, h, init, 1000); e1.record(); torch.cuda.synchronize()
print("after 2 s idle", round(e0.elapsed_time(e1), 3))
