"""Per-step latency of the fused Ant rollout under different weight patterns (zero, one
random policy copied to every row, independent random rows) at several populations."""
import sys, time, torch
sys.path.insert(0, "/root/repo")
from evoxmi import random as rnd
from evoxmi.ops import neuro
from evoxmi.problems.neuroevolution.reinforcement_learning.envs import get_environment

h = 64
P = neuro.ant_param_count(h, h)
s0, _ = get_environment("ant").reset(rnd.PRNGKey(0), 1)
init = s0[0].cuda()
g = torch.Generator(device="cuda").manual_seed(0)
from evoxmi.models import MLPPolicy
from evoxmi.utils import TreeAndVector
pol = MLPPolicy([27, h, h, 8])
center = TreeAndVector(pol.init(rnd.PRNGKey(0), device="cuda")).to_vector(pol.init(rnd.PRNGKey(0), device="cuda"))
modes = sys.argv[1].split(",") if len(sys.argv) > 1 else ["zero", "same", "random", "random_x0.02", "es", "es_x0.5"]
for pop in (64, 512, 1024):
    for mode in modes:
        if mode.startswith("file:"):
            W = torch.load(mode[5:], weights_only=True).cuda()
            half = mode.endswith("#half")
            W = W[: W.shape[0] // 2] if half else W
            if W.shape[0] != pop:
                continue
        elif mode.startswith("es"):
            sig = 0.05 * (10 if mode.endswith("0.5") else 1)
            W = center[None, :] + sig * torch.randn(pop, P, device="cuda", generator=g)
        elif mode == "zero":
            W = torch.zeros(pop, P, device="cuda")
        elif mode == "same":
            W = (0.1 * torch.randn(1, P, device="cuda", generator=g)).expand(pop, P).contiguous()
        else:
            sc = 0.02 if mode.endswith("0.02") else 0.1
            W = sc * torch.randn(pop, P, device="cuda", generator=g)
        _, st = neuro.ant_rollout(W, h, h, init, 1000)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            _, st = neuro.ant_rollout(W, h, h, init, 1000)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        mx = int(st.max())
        print(f"pop {pop:5d} {mode:12s} {ms:8.3f} ms  max_len {mx:5d} mean_len {float(st.float().mean()):7.1f}  us/step(longest) {1e3 * ms / max(mx, 1):.3f}", flush=True)
