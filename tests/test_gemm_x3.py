"""gemm_ks bf16x3 products (PREC 3) and the diagonal-add epilogue (csrc/kernels/gemm_ks.hip):
the eigensolver's correction products, checked against an fp64 torch reference of the same op.
bf16x3 keeps ≈16 bits: |C − C_ref| ≤ 4e-5·Σ|ab| (the f32-accurate modes keep 2e-6)."""
import pytest
import torch

from evoxmi.ops import linalg


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_diag_add_semantics(device):
    g = torch.Generator().manual_seed(1)
    T = torch.randn(64, 64, generator=g).to(device)
    out = torch.empty(64, 64, device=device)
    linalg.mm(T, T, ta=True, mode=1, out=out, diag_add=-1.0)
    R = T.double().t() @ T.double() - torch.eye(64, dtype=torch.float64, device=device)
    assert torch.allclose(out.double(), R, atol=1e-4 * float(R.abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,ta,tb", [(1000, 1000, 1000, False, True), (1000, 1000, 1000, False, False),
                                         (1000, 1000, 1000, True, False), (200, 130, 36, False, False),
                                         (64, 1000, 1000, False, False), (1000, 125, 1000, False, True)])
def test_gemm_x3_bound(M, N, K, ta, tb):
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(*((K, M) if ta else (M, K)), generator=g)
    B = torch.randn(*((N, K) if tb else (K, N)), generator=g)
    Am, Bm = (A.t() if ta else A).double(), (B.t() if tb else B).double()
    out = torch.empty(M, N, device="cuda")
    linalg.mm(A.cuda(), B.cuda(), ta=ta, tb=tb, out=out, prec="x3")
    err = (out.cpu().double() - Am @ Bm).abs()
    S = Am.abs() @ Bm.abs()
    assert (err <= 4e-5 * S + 1e-30).all(), float((err / S).max())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1000, 332])
def test_gemm_x3_symmetric_and_skew_outputs(n):
    """X² = −X·Xᵀ (mode 1) and X³ = −X²·Xᵀ (mode 2) for a skew X: the eigensolver's Taylor terms."""
    g = torch.Generator().manual_seed(n)
    S = torch.randn(n, n, generator=g)
    X = (S - S.t()).contiguous()
    X2 = torch.empty(n, n, device="cuda")
    linalg.mm(X.cuda(), X.cuda(), tb=True, mode=1, alpha=-1.0, out=X2, prec="x3")
    R2 = -(X.double() @ X.double().t())
    S2 = X.double().abs() @ X.double().abs().t()
    assert ((X2.cpu().double() - R2).abs() <= 4e-5 * S2).all()
    assert torch.equal(X2, X2.t())
    X3 = torch.empty(n, n, device="cuda")
    X2f = R2.float().cuda()
    linalg.mm(X2f, X.cuda(), tb=True, mode=2, alpha=-1.0, out=X3, prec="x3")
    R3 = -(R2.float().double() @ X.double().t())
    S3 = R2.float().double().abs() @ X.double().abs().t()
    assert ((X3.cpu().double() - R3).abs() <= 4e-5 * S3 + 1e-30).all()
    assert torch.equal(X3, -X3.t())


@pytest.mark.gpu
def test_gemm_x3_correction_plus_exact_base():
    """B + B·(V − I) with ‖V − I‖ ≈ 1e-3: the x3 correction product leaves the sum f32-accurate
    (error ≤ 1e-7·|B|) — the form the eigensolver's basis update uses."""
    g = torch.Generator().manual_seed(3)
    n = 1000
    Bq, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    X = 1e-3 * torch.randn(n, n, generator=g, dtype=torch.float64) / n ** 0.5
    X = X - X.t()
    Vm = torch.linalg.matrix_exp(X) - torch.eye(n, dtype=torch.float64)  # V − I
    Bf, Vf = Bq.float().contiguous(), Vm.float().contiguous()
    out = torch.empty(n, n, device="cuda")
    # Vᵀ stored (the eigensolver's VT layout): B·V = mm(Bq, VT, tb=True)
    VT = Vf.t().contiguous()
    linalg.mm(Bf.cuda(), VT.cuda(), tb=True, beta=1.0, Cin=Bf.cuda(), out=out, prec="x3")
    R = Bf.double() + Bf.double() @ Vf.double()
    assert float((out.cpu().double() - R).abs().max()) <= 1e-7 * float(Bq.abs().max())
