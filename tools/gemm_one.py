import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evoxmi.ops import _ext
from evoxmi.ops.linalg import Operand, gemm
ops = _ext.ops()
cfg = int(os.environ.get("CFG", "1"))
ops.gemm_set_config(cfg)
dev = torch.device("cuda")
A = torch.randn(10000, 1000, device=dev)
B = torch.randn(1000, 1000, device=dev)
D = torch.rand(1000, device=dev)
for _ in range(5):
    gemm(Operand(A), Operand(B), 10000, 1000, 1000)
    gemm(Operand(A, kscale=D), Operand(B), 10000, 1000, 1000)
    A @ B.T
torch.cuda.synchronize()
