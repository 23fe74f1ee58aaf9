"""gemm_sq (csrc/kernels/gemm_sq.hip): the opt-in LDS-staged bf16x6 kernel that evx_gemm_ks
routes square products to when enabled (measured slower than gemm_ks: off by default).  Against an fp64 reference at gemm_ks's
2e-6·Σ|a·b| bound and against gemm_ks itself (forced with a tile override): every operand
layout, K tails inside a 16-k stage, the (skew-)symmetric upper-tile mode with its mirror and
stats partials, and the device-selected A2 / α2 / C2 variant."""
import pytest
import torch

from evoxmi.ops import _ext, linalg

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _sq_on():
    _ext.ops().gemm_sq_enable(1)
    yield
    _ext.ops().gemm_sq_enable(0)


def _ref(A, B, ta, tb):
    return (A.t() if ta else A).double() @ (B.t() if tb else B).double()


def _tol(A, B, ta, tb):
    return 2e-6 * ((A.t() if ta else A).double().abs() @ (B.t() if tb else B).double().abs()) + 1e-30


class _ForceKs:
    """gemm_ks with its own tile heuristic (a tile override disables the gemm_sq route)."""

    def __enter__(self):
        _ext.ops().gemm_ks_set_tile(4)

    def __exit__(self, *a):
        _ext.ops().gemm_ks_set_tile(0)


@pytest.mark.parametrize("M,N,K", [(1000, 1000, 1000), (256, 512, 100), (1000, 1000, 4), (640, 128, 20), (1000, 1000, 2048)])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
def test_gemm_sq_matches_fp64_and_gemm_ks(M, N, K, ta, tb):
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K + 2 * ta + tb)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((N, K) if tb else (K, N), generator=g)
    assert _ext.ops().gemm_ks_grid(M, N, 0) == -(-M // 64) * -(-N // 64)  # routed to gemm_sq
    C = linalg.mm(A.cuda(), B.cuda(), ta=ta, tb=tb).cpu().double()
    R = _ref(A, B, ta, tb)
    assert ((C - R).abs() <= _tol(A, B, ta, tb)).all(), float((C - R).abs().max())
    with _ForceKs():
        Ck = linalg.mm(A.cuda(), B.cuda(), ta=ta, tb=tb).cpu().double()
    assert ((C - Ck).abs() <= 2 * _tol(A, B, ta, tb)).all()


@pytest.mark.parametrize("n,K", [(1000, 1000), (200, 36), (128, 1000)])
def test_gemm_sq_symmetric_skew_and_stats(n, K):
    g = torch.Generator().manual_seed(n + K)
    Y = torch.randn(K, n, generator=g)
    ops = _ext.ops()
    nparts = int(ops.gemm_ks_grid(n, n, 1))
    assert nparts == (n // 64 + (n % 64 > 0)) * (n // 64 + (n % 64 > 0) + 1) // 2
    part = torch.full((4 * nparts,), float("nan"), dtype=torch.float64, device="cuda")
    S = linalg.mm(Y.cuda(), Y.cuda(), ta=True, mode=1, stat_part=part, out=torch.empty(n, n, device="cuda")).cpu()
    R = Y.double().t() @ Y.double()
    assert torch.equal(S, S.t())
    assert ((S.double() - R).abs() <= _tol(Y, Y, True, False)).all()
    p = part.view(-1, 4).cpu()
    assert torch.isfinite(p).all()  # every workgroup wrote its partial
    Sd = S.double()
    dg = torch.diagonal(Sd)
    off = (Sd * Sd).sum() - (dg * dg).sum()
    assert torch.allclose(p[:, 0].sum(), off, rtol=1e-6)
    assert torch.allclose(p[:, 1].sum(), (dg * dg).sum(), rtol=1e-9)
    assert float(p[:, 2].min()) == float(dg.min()) and float(p[:, 3].max()) == float(dg.max())
    # diagonal-only stats (the eigensolver's X² bounds)
    part.fill_(float("nan"))
    linalg.mm(Y.cuda(), Y.cuda(), ta=True, mode=1, stat_part=part, stat_diag_only=True, out=torch.empty(n, n, device="cuda"))
    p = part.view(-1, 4).cpu()
    assert torch.isfinite(p).all() and float(p[:, 0].sum()) == 0.0
    assert torch.allclose(p[:, 1].sum(), (dg * dg).sum(), rtol=1e-9)
    if n == K:
        X = torch.randn(n, n, generator=g)
        X = (X - X.t()) / 2
        X2f = (X.double() @ X.double()).float()
        X3 = linalg.mm(X2f.cuda(), X.cuda(), tb=True, mode=2, alpha=-1.0).cpu()
        assert torch.equal(X3, -X3.t())
        R3 = X2f.double() @ X.double()
        assert ((X3.double() - R3).abs() <= _tol(X2f, X, False, False)).all()


def test_gemm_sq_device_selected_variant_and_epilogue():
    """sel = 0: α·A·Bᵀ + β·Cin into C; sel = 1: α2·A2·Bᵀ + β·Cin into C2 (the eigensolver's
    order-4 / order-6 Taylor product and the Newton–Schulz output switch), bias, *α, skip."""
    g = torch.Generator().manual_seed(9)
    n = 1000
    A, A2, B = (torch.randn(n, n, generator=g).cuda() for _ in range(3))
    Cin = torch.randn(n, n, generator=g).cuda()
    bias = torch.randn(n, generator=g).cuda()
    ap = torch.tensor([0.5], device="cuda")
    for s in (0, 1):
        sel = torch.full((1,), s, dtype=torch.int32, device="cuda")
        C = torch.full((n, n), 7.0, device="cuda")
        C2 = torch.full((n, n), 7.0, device="cuda")
        linalg.mm(A, B, tb=True, alpha=2.0, alpha_ptr=ap, bias_n=bias, beta=-1.0, Cin=Cin, out=C, sel=sel, A2=A2, alpha2=-3.0, C2=C2)
        Ause, a, tgt, other = (A, 2.0, C, C2) if s == 0 else (A2, -3.0, C2, C)
        R = a * 0.5 * _ref(Ause.cpu(), B.cpu(), False, True) + bias.cpu().double() - Cin.cpu().double()
        tol = abs(a) * 0.5 * _tol(Ause.cpu(), B.cpu(), False, True) + 1e-5
        assert ((tgt.cpu().double() - R).abs() <= tol).all()
        assert bool((other == 7.0).all())
    skip = torch.ones(1, dtype=torch.int32, device="cuda")
    C = torch.full((n, n), 7.0, device="cuda")
    linalg.mm(A, B, tb=True, out=C, skip=skip)
    assert bool((C == 7.0).all())


def test_gemm_sq_is_deterministic_and_in_place():
    g = torch.Generator().manual_seed(5)
    A, B = torch.randn(1000, 1000, generator=g).cuda(), torch.randn(1000, 1000, generator=g).cuda()
    assert torch.equal(linalg.mm(A, B), linalg.mm(A, B))
    out = torch.randn(1000, 1000, generator=g).cuda()
    ref = _ref(A.cpu(), B.cpu(), False, True) + out.cpu().double()
    linalg.mm(A, B, tb=True, beta=1.0, Cin=out, out=out)
    assert ((out.cpu().double() - ref).abs() <= _tol(A.cpu(), B.cpu(), False, True) + 1e-5).all()
