"""With EVOXMI_ANT_TRACE=1 the rollout returns per-wave shader cycles and HW_ID/XCC_ID: wave
placement (waves per SIMD) and cycles of the longest waves, with and without a 26 MB
elementwise kernel right before the launch."""
import collections, sys, torch
sys.path.insert(0, "/root/repo")
from evoxmi import random as rnd
from evoxmi.ops import neuro
from evoxmi.problems.neuroevolution.reinforcement_learning.envs import get_environment

W = torch.load(sys.argv[1], weights_only=True).cuda()
s0 = get_environment("ant").reset(rnd.PRNGKey(0), 1)[0][0].cuda()
x = torch.randn(W.numel(), device="cuda")
for tag in ("nothing", "elementwise", "nothing", "elementwise"):
    if tag == "elementwise":
        x.mul_(1.0000001)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    cyc, hw = neuro.ant_rollout(W, 64, 64, s0, 1000)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    hw = hw.cpu().tolist()
    cyc = cyc.cpu()
    simd = collections.Counter((h >> 16, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 15, (h >> 4) & 3) for h in hw)
    cu = collections.Counter((h >> 16, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 15) for h in hw)
    print(f"{tag:12s} {ms:7.2f} ms  max cycles {float(cyc.max()):.3e} (={float(cyc.max()) / ms / 1e6:.2f} GHz if max wave spans the kernel)"
          f"  median {float(cyc.median()):.3e}  SIMDs used {len(simd)}  waves/SIMD hist {sorted(collections.Counter(simd.values()).items())}"
          f"  CUs used {len(cu)} waves/CU hist {sorted(collections.Counter(cu.values()).items())}", flush=True)
