"""Rollout time of a saved evolved population after idle time and after each import."""
import importlib, sys, time, torch
sys.path.insert(0, "/root/repo")
from evoxmi import random as rnd
from evoxmi.ops import neuro
from evoxmi.problems.neuroevolution.reinforcement_learning.envs import get_environment

W = torch.load(sys.argv[1], weights_only=True).cuda()
s0 = get_environment("ant").reset(rnd.PRNGKey(0), 1)[0][0].cuda()


def t(tag, n=2):
    out = []
    for _ in range(n):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        neuro.ant_rollout(W, 64, 64, s0, 1000)
        e1.record()
        torch.cuda.synchronize()
        out.append(round(e0.elapsed_time(e1), 2))
    print(f"{tag:34s} {out}", flush=True)


t("fresh", 3)
time.sleep(1.5)
t("after 1.5 s idle")
x = torch.randn(4096, 4096, device="cuda")
t0 = time.time()
while time.time() - t0 < 1.0:
    x = x * 1.0001
t("after 1 s of small kernels")
for m in ["evoxmi.utils", "evoxmi.models", "evoxmi.algorithms", "evoxmi.workflows", "evoxmi.problems.neuroevolution"]:
    t0 = time.time()
    importlib.import_module(m)
    t(f"import {m} ({time.time() - t0:.2f}s)")
