import torch
from evoxmi import random as rnd
from evoxmi.algorithms import CMAES
from evoxmi.ops import sbr_device
from evoxmi.problems.numerical import CEC2022TestSuit
from evoxmi.workflows import StdWorkflow
orig = sbr_device.DeviceSBR.solve
n_solve = [0]
def hooked(ws, C, B_prev, *a, **k):
    if n_solve[0] + 1 in (10, 40, 41):
        torch.save({"C": C.detach().cpu().clone(), "B_prev": B_prev.detach().cpu().clone()}, f"gpurun_out/dl/mat_{n_solve[0] + 1}.pt")
    out = orig(ws, C, B_prev, *a, **k)
    torch.cuda.synchronize()
    h = ws.hist.view(-1, 4).cpu()
    off, dg, mn, mx = h[:, 0].clamp(min=0), h[:, 1], h[:, 2], h[:, 3]
    r = (off / dg).sqrt(); kap = off.sqrt() / (mx - mn)
    n = int(ws.st[2].item())
    ctrl = ws.ctrl.view(-1, 8).cpu()
    n_solve[0] += 1
    line = f"solve {n_solve[0]:3d} K {ws.K} lean {ws.lean_from} iters {n}: r " + " ".join(f"{float(r[j]):.1e}" for j in range(n + 1))
    line += " | far " + "".join("F" if int(ctrl[j][1]) == 0 else "n" for j in range(n))
    line += " | ord6 " + "".join(str(int(ctrl[j][4])) for j in range(n))
    line += " | ns " + "".join("1" if int(ctrl[j][5]) == 0 else "0" for j in range(n))
    line += " | a " + " ".join(f"{float(ws.alpha[j+1].item()):.2f}" for j in range(n))
    line += " | theta " + "".join(str(int(ws.theta[j].item())) for j in range(n))
    print(line, flush=True)
    return out
sbr_device.DeviceSBR.solve = hooked
center = (torch.rand(1000, generator=torch.Generator().manual_seed(1)) * 160 - 80).cuda()
algo = CMAES(center_init=center, init_stdev=20.0, pop_size=10000)
wf = StdWorkflow(algo, CEC2022TestSuit.create(1), graph=False)
st = wf.init(rnd.PRNGKey(2024, device=torch.device("cuda")))
for g in range(42):
    st = wf.step(st)
