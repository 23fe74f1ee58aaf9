"""Rollout time (evolved population, pop 1024) when each call is preceded by different work:
nothing, a tiny kernel, a 26 MB elementwise pass (the OpenES ask's population build), a
compute-bound GEMM, or host idle time."""
import sys, time, torch
sys.path.insert(0, "/root/repo")
from evoxmi import random as rnd
from evoxmi.ops import neuro
from evoxmi.problems.neuroevolution.reinforcement_learning.envs import get_environment

W = torch.load(sys.argv[1], weights_only=True).cuda()
s0 = get_environment("ant").reset(rnd.PRNGKey(0), 1)[0][0].cuda()
x = torch.randn(W.numel(), device="cuda")
a = torch.randn(2048, 2048, device="cuda")


def run(tag, pre, n=4):
    out = []
    for _ in range(n):
        pre()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        neuro.ant_rollout(W, 64, 64, s0, 1000)
        e1.record()
        torch.cuda.synchronize()
        out.append(round(e0.elapsed_time(e1), 2))
    print(f"{tag:28s} {out}", flush=True)


def nothing():
    pass


def tiny():
    x[:16].add_(1.0)


def stream26():
    x.mul_(1.0000001)


def stream26x4():
    for _ in range(4):
        x.mul_(1.0000001)


def gemm():
    torch.mm(a, a)


def idle():
    torch.cuda.synchronize()
    time.sleep(0.005)


for tag, f in [("nothing", nothing), ("tiny kernel", tiny), ("26 MB elementwise", stream26), ("4x 26 MB elementwise", stream26x4),
               ("2048^3 GEMM", gemm), ("5 ms host idle", idle), ("nothing (again)", nothing)]:
    run(tag, f)
