"""Same rollout (an evolved population saved by bench_neuro --dump-pop) timed after each stage
of building an OpenES workflow in one process: which stage makes the kernel slower?"""
import sys, time, torch
sys.path.insert(0, "/root/repo")
from evoxmi import random as rnd
from evoxmi.ops import neuro
from evoxmi.problems.neuroevolution.reinforcement_learning.envs import get_environment

W = torch.load(sys.argv[1], weights_only=True).cuda()
s0 = get_environment("ant").reset(rnd.PRNGKey(0), 1)[0][0].cuda()


def t(tag):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _, L = neuro.ant_rollout(W, 64, 64, s0, 1000)
    e1.record()
    torch.cuda.synchronize()
    print(f"{tag:28s} {e0.elapsed_time(e1):8.3f} ms  mean_len {float(L.float().mean()):.1f}", flush=True)


t("fresh")
t("fresh again")
from evoxmi.algorithms import OpenES
from evoxmi.models import MLPPolicy
from evoxmi.problems.neuroevolution import Brax
from evoxmi.utils import TreeAndVector, rank_based_fitness
from evoxmi.workflows import StdWorkflow
t("after imports")
policy = MLPPolicy([27, 64, 64, 8])
params = policy.init(rnd.PRNGKey(0), device="cuda")
tv = TreeAndVector(params)
algo = OpenES(tv.to_vector(params), 1024, learning_rate=0.01, noise_stdev=0.05, optimizer="adam")
prob = Brax(policy, "ant", 1000)
wf = StdWorkflow(algo, prob, sol_transforms=[tv.batched_to_tree], fit_transforms=[rank_based_fitness], opt_direction="max")
st = wf.init(rnd.PRNGKey(1, device="cuda"))
t("after wf.init")
for g in range(6):
    st = wf.step(st)
    t(f"after gen {g}")
big = torch.empty(int(2e9), dtype=torch.uint8, device="cuda")
t("after +2 GB alloc")
del big
torch.cuda.empty_cache()
t("after empty_cache")
