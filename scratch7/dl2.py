import torch, math
torch.set_printoptions(precision=3, linewidth=220, threshold=100000)
from evoxmi import random as rnd
from evoxmi.algorithms import CMAES
from evoxmi.ops import sbr_device
from evoxmi.problems.numerical import CEC2022TestSuit
from evoxmi.workflows import StdWorkflow

orig = sbr_device.eigh_device
calls = []
def hooked(C, B_prev, *a, **k):
    out = orig(C, B_prev, *a, **k)
    torch.cuda.synchronize()
    ws = [w for w in sbr_device._WS.values() if w.K == 32][0]
    h = ws.hist.view(-1, 4).cpu()
    off, dg, mn, mx = h[:, 0].clamp(min=0), h[:, 1], h[:, 2], h[:, 3]
    r = (off / dg).sqrt(); kap = off.sqrt() / (mx - mn)
    n = int(ws.st[2].item())
    ctrl = ws.ctrl.view(-1, 8).cpu()
    calls.append(1)
    st = out[2].cpu() if isinstance(out[2], torch.Tensor) else out[2]
    print(f"solve {len(calls)} iters {n} stats {st.tolist() if hasattr(st,'tolist') else st} spread {float(mn[0]):.3e}..{float(mx[0]):.3e}")
    for j in range(n + 1):
        c = ctrl[j].tolist() if j < n else None
        print(f"   j{j-1:3d} r {float(r[j]):.3e} kappa {float(kap[j]):.3e} alpha {float(ws.alpha[j].item()):.3f} theta {float(ws.theta[min(j,ws.K-1)].item()):.2f} ctrl {c}")
    return out
sbr_device.eigh_device = hooked
center = (torch.rand(1000, generator=torch.Generator().manual_seed(2)) * 160 - 80).cuda()
algo = CMAES(center_init=center, init_stdev=20.0)
wf = StdWorkflow(algo, CEC2022TestSuit.create(1), graph=False)
st = wf.init(rnd.PRNGKey(2024, device=torch.device("cuda")))
for g in range(56):
    st = wf.step(st)
