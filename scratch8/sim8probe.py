import hashlib, sys, torch
sys.path.insert(0, ".")
from evoxmi import random as rnd
from evoxmi.algorithms import CMAES
from evoxmi.ops import sbr_device
from evoxmi.parallel.context import SimulatedDistContext
from evoxmi.problems.numerical import CEC2022TestSuit
from evoxmi.workflows import StdWorkflow
torch.set_printoptions(linewidth=200, precision=3)
center = (torch.rand(1000, generator=torch.Generator().manual_seed(1)) * 160 - 80).cuda()
algo = CMAES(center_init=center, init_stdev=20.0, pop_size=10000)
wf = StdWorkflow(algo, CEC2022TestSuit.create(1), graph=False)
st = wf.init(rnd.PRNGKey(2024, device=torch.device("cuda")))
st = wf.enable_distributed(st, context=SimulatedDistContext(0, 8, algorithm=algo))
snap = sbr_device.snapshot_counts()
hs = []
for g in range(14):
    st = wf.step(st)
    torch.cuda.synchronize()
    m = st.get_child_state("algorithm").mean
    hs.append(hashlib.sha1(m.cpu().numpy().tobytes()).hexdigest()[:8])
h = sbr_device.histories_since(snap)
print(sys.argv[1], " ".join(hs))
print(h[:, :3].T)
