"""Per-sweep cost of the SBR block kernel (sweeps = 0 isolates sort + gather + store)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evoxmi.ops import _ext  # noqa: E402

ops = _ext.ops()
for n in (1000, 256):
    A = torch.randn(n, n, device="cuda")
    A = A + A.T
    for sw in (0, 1, 2, 4):
        ops.sbr_block(A, 0, sw)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            ops.sbr_block(A, 0, sw)
        e.record()
        torch.cuda.synchronize()
        print(f"n={n} sweeps={sw}: {s.elapsed_time(e) / 10 * 1e3:.1f} us", flush=True)

A = torch.randn(1000, 1000, device="cuda")
A = A + A.T
for probe in (0, 1, 2, 3):
    dbg = torch.zeros(3 * 16, dtype=torch.int64, device="cuda")
    ops.sbr_block(A, 0, 2 + (probe << 8), dbg)
    torch.cuda.synchronize()
    d = dbg.view(16, 3).cpu()
    print("probe %d cycles per round: phaseA %.0f phaseB %.0f total-loop %.0f" % (probe, d[:, 0].float().mean() / 126, d[:, 1].float().mean() / 126, d[:, 2].float().mean() / 126))

# version-2 kernel (sbr_block2_kernel) variants: per-call time at sweeps = 2
names = {8: "v2 full", 9: "v2 no Q", 10: "v2 no S blocks", 11: "v2 rotations only", 12: "v2 one rotation/thread",
         13: "v2 one rotation, no Q", 15: "v2 one rotation only", 4: "v1"}
for probe in (8, 9, 10, 11, 12, 13, 15, 4):
    ops.sbr_block(A, 0, 2 + (probe << 8))
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        ops.sbr_block(A, 0, 2 + (probe << 8))
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / 10 * 1e3
    print(f"{names[probe]}: {t:.1f} us = {t * 2.4e3 / 126:.0f} cycles/round", flush=True)
