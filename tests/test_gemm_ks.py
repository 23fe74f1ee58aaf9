"""gemm_ks (csrc/kernels/gemm_ks.hip): the flagship's f32 MFMA GEMM vs an fp64 torch
reference of the same product, over operand layouts, output modes (full / symmetric /
skew-symmetric), K tails, ragged M/N edges and the fused epilogue."""
import pytest
import torch

from evoxmi import config
from evoxmi.ops import linalg

PRECS = ["x6", "x6w", "f32"]  # bf16x6 split products on 16x16x32 / 32x32x16 MFMA, and the f32 MFMA path


def _ref(A, B, ta, tb, alpha=1.0, bias=None, beta=0.0, Cin=None):
    Am = (A.t() if ta else A).double()
    Bm = (B.t() if tb else B).double()
    C = alpha * (Am @ Bm)
    if bias is not None:
        C = C + bias.double()[None, :]
    if Cin is not None:
        C = C + beta * Cin.double()
    return C


def test_mm_cpu_semantics():
    g = torch.Generator().manual_seed(0)
    A, B = torch.randn(7, 12, generator=g), torch.randn(9, 12, generator=g)
    C = linalg.mm(A, B, tb=True, alpha=2.0, bias_n=torch.ones(9))
    assert torch.allclose(C.double(), _ref(A, B, False, True, 2.0, torch.ones(9)), atol=1e-5)
    C = linalg.mm(A.t().contiguous(), B.t().contiguous(), ta=True)
    assert torch.allclose(C.double(), _ref(A, B, False, True), atol=1e-5)


def _tol(A, B, ta, tb, K):
    # f32 fmaf chains: error ≈ 1e-7·Σ|a·b| for random signs, more on same-sign sums (the
    # diagonal of a Gram matrix); 2e-6·Σ|a·b| still rejects any wrong term
    Am = (A.t() if ta else A).double().abs()
    Bm = (B.t() if tb else B).double().abs()
    return 2e-6 * (Am @ Bm) + 1e-30


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1000, 1000, 1000), (257, 130, 72), (64, 48, 20), (1000, 1000, 5000), (333, 1000, 1000),
                                   (10000, 1000, 1000)])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("prec", PRECS)
def test_gemm_ks_full_matches_fp64(M, N, K, ta, tb, prec):
    if M * N * K > 2e9 and (ta, tb) != (False, True):
        pytest.skip("large shape: the NT layout only")
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K + 2 * ta + tb)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((N, K) if tb else (K, N), generator=g)
    with config.override(gemm_prec=prec):
        C = linalg.mm(A.cuda(), B.cuda(), ta=ta, tb=tb).cpu().double()
    R = _ref(A, B, ta, tb)
    assert ((C - R).abs() <= _tol(A, B, ta, tb, K)).all(), float((C - R).abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("n,K", [(1000, 1000), (1000, 5000), (200, 36), (48, 16), (97, 1000)])
@pytest.mark.parametrize("prec", PRECS)
def test_gemm_ks_symmetric_and_skew_outputs(n, K, prec):
    with config.override(gemm_prec=prec):
        _sym_skew(n, K)


def _sym_skew(n, K):
    g = torch.Generator().manual_seed(n + K)
    Y = torch.randn(K, n, generator=g)
    # symmetric: Yᵀ Y (both operands RC) and Z Zᵀ (both KC)
    S = linalg.mm(Y.cuda(), Y.cuda(), ta=True, mode=1).cpu()
    R = Y.double().t() @ Y.double()
    assert torch.equal(S, S.t())
    assert ((S.double() - R).abs() <= _tol(Y, Y, True, False, K)).all()
    Z = Y.t().contiguous()
    S2 = linalg.mm(Z.cuda(), Z.cuda(), tb=True, mode=1).cpu()
    assert torch.equal(S2, S2.t()) and ((S2.double() - R).abs() <= _tol(Z, Z, False, True, K)).all()
    if n == K:
        # skew: X² X = −X² Xᵀ for skew X (the Taylor chain of the eigensolver)
        X = torch.randn(n, n, generator=g)
        X = (X - X.t()) / 2
        X2 = X.double() @ X.double()
        X2f = X2.float()
        X3 = linalg.mm(X2f.cuda(), X.cuda(), tb=True, mode=2, alpha=-1.0).cpu()
        assert torch.equal(X3, -X3.t())
        R3 = X2f.double() @ X.double()
        assert ((X3.double() - R3).abs() <= _tol(X2f, X, False, False, n)).all()


@pytest.mark.gpu
def test_gemm_ks_epilogue_alpha_ptr_bias_cin_out_and_skip():
    g = torch.Generator().manual_seed(11)
    M, N, K = 1000, 1000, 1000
    A, B = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    bias, Cin = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    ap = torch.tensor([0.75])
    C = linalg.mm(A.cuda(), B.cuda(), tb=True, alpha=2.0, alpha_ptr=ap.cuda(), bias_n=bias.cuda(), beta=-0.5, Cin=Cin.cuda())
    R = _ref(A, B, False, True, 1.5, bias, -0.5, Cin)
    assert ((C.cpu().double() - R).abs() <= 1.5 * _tol(A, B, False, True, K) + 1e-6).all()
    # in place (Cin may alias out: every element is read before it is written by its owner)
    out = Cin.clone().cuda()
    linalg.mm(A.cuda(), B.cuda(), tb=True, beta=1.0, Cin=out, out=out)
    R = _ref(A, B, False, True, 1.0, None, 1.0, Cin)
    assert ((out.cpu().double() - R).abs() <= _tol(A, B, False, True, K) + 1e-6).all()
    # skip word: nothing written while it is non-zero
    sentinel = torch.full((M, N), 7.0, device="cuda")
    skip = torch.ones(1, dtype=torch.int32, device="cuda")
    linalg.mm(A.cuda(), B.cuda(), tb=True, out=sentinel, skip=skip)
    assert bool((sentinel == 7.0).all())
    skip.zero_()
    linalg.mm(A.cuda(), B.cuda(), tb=True, out=sentinel, skip=skip)
    assert ((sentinel.cpu().double() - _ref(A, B, False, True)).abs() <= _tol(A, B, False, True, K)).all()


@pytest.mark.gpu
def test_gemm_x6_scaled_and_mixed_magnitude_operands():
    """bf16x6 keeps f32 accuracy over operand magnitudes spanning many binades (each part is
    split relative to its own value, so no shared exponent is assumed): rows scaled by
    10^-20 … 10^20 and columns of mixed sign and size."""
    g = torch.Generator().manual_seed(3)
    A = torch.randn(300, 256, generator=g) * torch.logspace(-20, 20, 300)[:, None]
    B = torch.randn(200, 256, generator=g) * torch.logspace(-3, 3, 256)[None, :]
    with config.override(gemm_prec="x6"):
        C = linalg.mm(A.cuda(), B.cuda(), tb=True).cpu().double()
    R = _ref(A, B, False, True)
    assert ((C - R).abs() <= _tol(A, B, False, True, 256)).all()


@pytest.mark.gpu
def test_gemm_ks_is_deterministic():
    g = torch.Generator().manual_seed(5)
    A, B = torch.randn(1000, 1000, generator=g).cuda(), torch.randn(1000, 1000, generator=g).cuda()
    C1 = linalg.mm(A, B)
    C2 = linalg.mm(A, B)
    assert torch.equal(C1, C2)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(10000, 1000, 1000), (300, 200, 100), (32, 5120, 20)])
def test_gemm_ks_fused_shift_prologue(M, N, K):
    """z = s·(X − o)·Mᵀ with the shift fused into the A loads (CEC shift-rotate)."""
    g = torch.Generator().manual_seed(M + K)
    X, R = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    o = torch.randn(K, generator=g)
    Z = linalg.mm(X.cuda(), R.cuda(), tb=True, alpha=0.5, a_sub_k=o.cuda()).cpu().double()
    ref = 0.5 * ((X.double() - o.double()) @ R.double().t())
    tol = 2e-6 * 0.5 * ((X - o).double().abs() @ R.double().abs().t())
    assert ((Z - ref).abs() <= tol + 1e-30).all()
    # exact zero at the optimum (the shift happens before the products, as in the reference)
    Z0 = linalg.mm(o[None, :].repeat(4, 1).cuda(), R.cuda(), tb=True, a_sub_k=o.cuda())
    assert bool((Z0 == 0).all())


@pytest.mark.gpu
def test_gemm_per_block_shifts():
    """Stacked shifted products in one launch: column block c uses shift row c (exact zero when
    a row equals its block's shift)."""
    g = torch.Generator().manual_seed(9)
    M, K, blocks, W = 3000, 1000, 3, 1024
    X = torch.randn(M, K, generator=g)
    Bs = torch.randn(blocks * W, K, generator=g)
    O = torch.randn(blocks, K, generator=g)
    X[5] = O[1]
    Z = linalg.mm_nt(X.cuda(), Bs.cuda(), a_sub_k=O.cuda(), sub_cols=W).cpu().double()
    for c in range(blocks):
        ref = (X.double() - O[c].double()) @ Bs[c * W : (c + 1) * W].double().t()
        tol = 2e-6 * ((X - O[c]).double().abs() @ Bs[c * W : (c + 1) * W].double().abs().t())
        assert ((Z[:, c * W : (c + 1) * W] - ref).abs() <= tol + 1e-30).all(), c
    assert bool((Z[5, W : 2 * W] == 0).all())


@pytest.mark.gpu
@pytest.mark.parametrize("f", [9, 10, 11, 12])
def test_cec2022_composition_stacked_gemm_matches_per_component(f):
    """F9–F12 at the synthetic d = 1000: the one-GEMM stacked rotations give the per-component
    GEMM result (and the CPU fp32 evaluation)."""
    from evoxmi.problems.numerical import CEC2022TestSuit

    p = CEC2022TestSuit.create(f)
    X = torch.rand(300, 1000, generator=torch.Generator().manual_seed(f)) * 200 - 100
    with config.override(cec_stack=1):
        a, _ = p.evaluate(None, X.cuda())
    with config.override(cec_stack=0):
        b, _ = p.evaluate(None, X.cuda())
    ref, _ = p.evaluate(None, X)
    assert torch.allclose(a.cpu(), b.cpu(), rtol=1e-5, atol=1e-4)
    assert torch.allclose(a.cpu(), ref, rtol=2e-3, atol=1e-3)
