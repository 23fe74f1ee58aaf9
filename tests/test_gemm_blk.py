"""gemm_blk (csrc/kernels/gemm_blk.hip): the LDS-staged bf16x6 GEMM on blocked planes vs an
fp64 torch reference of the same product, at the 2e-6·Σ|a·b| bound of tests/test_gemm_ks.py
(ragged M / N edges, K tails inside the last 16-k block, fused shift / column scale in the
split pass, the Philox planes producer, σ and bias epilogue, in-place output)."""
import pytest
import torch

from evoxmi import random as rnd
from evoxmi.ops import linalg


FMTS = {"blk": (linalg.blk_planes, linalg.normal_blk_planes, linalg.mm_blk),
        "h3": (linalg.h3_planes, linalg.normal_h3_planes, linalg.mm_h3)}


def _tol(A, B):
    return 2e-6 * (A.double().abs() @ B.double().abs().t()) + 1e-30


def test_blk_cpu_semantics():
    g = torch.Generator().manual_seed(0)
    X, Y = torch.randn(9, 20, generator=g), torch.randn(7, 20, generator=g)
    o, cs = torch.randn(20, generator=g), torch.rand(20, generator=g)
    A = linalg.blk_planes(X, sub_k=o)
    B = linalg.blk_planes(Y, colscale=cs)
    bias = torch.randn(7, generator=g)
    C = linalg.mm_blk(A, B, alpha=2.0, alpha_ptr=torch.tensor([0.5]), bias_n=bias)
    R = 1.0 * (X - o).double() @ (Y * cs).double().t() + bias.double()
    assert torch.allclose(C.double(), R, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", sorted(FMTS))
@pytest.mark.parametrize("M,N,K", [(10000, 1000, 1000), (1, 1, 1), (700, 130, 20), (333, 1000, 37), (2560, 256, 16),
                                   (10240, 1024, 1008), (5000, 600, 1000), (321, 129, 17), (640, 256, 4096), (100, 64, 5000),
                                   # population shards of the flagship: the 160 × 128 / 64 × 128-tile launches
                                   (5000, 1000, 1000), (2500, 1000, 1000), (1250, 1000, 1000), (1111, 520, 999)])
def test_gemm_blk_matches_fp64(M, N, K, fmt):
    split, _, mm = FMTS[fmt]
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g)
    sig = torch.tensor([0.75])
    Ap, Bp = split(A.cuda()), split(B.cuda())
    C = mm(Ap, Bp, alpha=2.0, alpha_ptr=sig.cuda(), bias_n=bias.cuda()).cpu().double()
    R = 1.5 * (A.double() @ B.double().t()) + bias.double()[None, :]
    err = (C - R).abs()
    assert (err <= 1.5 * _tol(A, B) + 1e-6 * bias.double().abs()[None, :]).all(), float(err.max())


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", sorted(FMTS))
def test_gemm_blk_fused_shift_scale_and_out(fmt):
    split, _, mm = FMTS[fmt]
    g = torch.Generator().manual_seed(5)
    M, N, K = 3000, 1000, 1000
    X = torch.randn(M, K, generator=g) * 80
    o = torch.randn(K, generator=g) * 80
    Bm = torch.randn(N, K, generator=g)
    D = torch.rand(K, generator=g) + 0.5
    out = torch.full((M + 5, N + 3), float("nan")).cuda()
    C = mm(split(X.cuda(), sub_k=o.cuda()), split(Bm.cuda(), colscale=D.cuda()), out=out[:M, :N])
    assert C.data_ptr() == out.data_ptr()
    A = (X - o).double()
    Bs = Bm.double() * D.double()
    R = A @ Bs.t()
    err = (C.cpu().double() - R).abs()
    assert (err <= 2e-6 * (A.abs() @ Bs.abs().t()) + 1e-30).all(), float(err.max())
    rest = out.cpu()
    assert torch.isnan(rest[M:, :]).all() and torch.isnan(rest[:, N:]).all()  # nothing written past M × N


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", sorted(FMTS))
@pytest.mark.parametrize("rows,d,row0", [(10000, 1000, 0), (130, 20, 7)])
def test_normal_blk_planes_match_the_noise_matrix(rows, d, row0, fmt):
    split, normal, mm = FMTS[fmt]
    key = rnd.PRNGKey(11, device="cuda")
    Z = rnd.normal(key, (rows, d), offset=row0 * d)
    I = torch.eye(d, device="cuda")
    # Z·I through the planes reproduces Z to the split's exactness (h + m + l = z exactly; the
    # six-product sum drops terms ≤ 2⁻²⁶|z|)
    C = mm(normal(key, rows, d, row0), split(I))
    # bf16x6: h + m + l = z exactly; f16x3: |z − h − m| ≤ 2⁻²²|z|
    assert torch.allclose(C, Z, rtol=1e-6 if fmt == "blk" else 6e-7, atol=1e-7 if fmt == "blk" else 1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", sorted(FMTS))
def test_gemm_blk_skip_word(fmt):
    split, _, mm = FMTS[fmt]
    A = split(torch.randn(400, 64, device="cuda"))
    B = split(torch.randn(200, 64, device="cuda"))
    out = torch.full((400, 200), 3.0, device="cuda")
    mm(A, B, out=out, skip=torch.ones(1, dtype=torch.int32, device="cuda"))
    assert (out == 3.0).all()
    mm(A, B, out=out, skip=torch.zeros(1, dtype=torch.int32, device="cuda"))
    assert not (out == 3.0).all()


@pytest.mark.gpu
def test_h3_row_scaling_keeps_relative_accuracy():
    """Rows of very different magnitude (per-row power-of-two scales), an all-zero row, and
    near-zero shifted rows (x ≈ o: the CEC rotation near the optimum) keep the fp64-referenced
    bound row by row."""
    g = torch.Generator().manual_seed(9)
    M, N, K = 700, 300, 1000
    mag = torch.logspace(-15, 15, M, dtype=torch.float64).float()
    X = torch.randn(M, K, generator=g) * mag[:, None]
    X[3] = 0.0
    Bm = torch.randn(N, K, generator=g) * torch.logspace(-4, 4, N, dtype=torch.float64).float()[:, None]
    C = linalg.mm_h3(linalg.h3_planes(X.cuda()), linalg.h3_planes(Bm.cuda())).cpu().double()
    R = X.double() @ Bm.double().t()
    tol = 2e-6 * (X.double().abs() @ Bm.double().abs().t()) + 1e-300
    assert ((C - R).abs() <= tol).all(), float(((C - R).abs() / tol).max())
    assert (C[3] == 0).all()
    # converged rows: x = o + 1e-4·ε, shifted in the split pass (the kernel's f32 x − o)
    o = torch.randn(K, generator=g) * 50
    Xc = o[None, :] + 1e-4 * torch.randn(64, K, generator=g)
    C = linalg.mm_h3(linalg.h3_planes(Xc.cuda(), sub_k=o.cuda()), linalg.h3_planes(Bm.cuda())).cpu().double()
    A = (Xc - o[None, :]).double()
    R = A @ Bm.double().t()
    tol = 2e-6 * (A.abs() @ Bm.double().abs().t()) + 1e-300
    assert ((C - R).abs() <= tol).all(), float(((C - R).abs() / tol).max())


@pytest.mark.gpu
def test_h3_tiny_and_wide_range_rows_stay_finite_and_bounded():
    """a row whose max is below ≈2⁻¹¹⁰ used to get a scale of 2^e > 2¹²⁸ = inf (NaN
    planes); the exponent is clamped.  A row spanning 20 decades keeps the Σ|ab| bound (its small
    elements fall into f16 subnormals of m, bounded absolutely by the row max)."""
    g = torch.Generator().manual_seed(11)
    M, N, K = 8, 64, 1000
    X = torch.randn(M, K, generator=g)
    X[0] *= 1e-36
    X[1] *= 5e-35
    X[2] = X[2] * torch.logspace(0, -20, K, dtype=torch.float64).float()
    X[3, :] = 0.0
    X[3, 17] = 1e-37
    Bm = torch.randn(N, K, generator=g)
    C = linalg.mm_h3(linalg.h3_planes(X.cuda()), linalg.h3_planes(Bm.cuda())).cpu().double()
    assert torch.isfinite(C).all()
    R = X.double() @ Bm.double().t()
    # f32 output resolution near the subnormal range: one ulp of the smallest normal
    tol = 2e-6 * (X.double().abs() @ Bm.double().abs().t()) + 2e-45
    assert ((C - R).abs() <= tol).all(), float(((C - R).abs() / tol).max())


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("M,K,ncomp,sub", [(700, 1000, 5, 1024), (333, 200, 3, 256), (64, 37, 2, 128), (1000, 1200, 2, 1280)])
def test_h3_stacked_components_match_fp64(device, M, K, ncomp, sub):
    """Stacked operands: one split of X into ncomp plane sets (x − o_c), one launch whose column
    block c uses set c — the composition functions' (x − o_c)·M_cᵀ for every component (K > 1024
    takes the per-component split passes)."""
    g = torch.Generator().manual_seed(M + K + ncomp)
    X = torch.randn(M, K, generator=g) * 50
    O = torch.randn(ncomp, K, generator=g) * 50
    Ms = torch.zeros(ncomp * sub, K)
    for c in range(ncomp):
        Ms[c * sub : c * sub + min(sub, K)] = torch.randn(min(sub, K), K, generator=g)
    Ap = linalg.h3_planes(X.to(device), sub_k=O.to(device))
    assert Ap.ncomp == ncomp
    C = linalg.mm_h3(Ap, linalg.h3_planes(Ms.to(device)), sub_cols=sub).cpu().double()
    assert C.shape == (M, ncomp * sub)
    for c in range(ncomp):
        A = (X - O[c]).double()
        Bc = Ms[c * sub : (c + 1) * sub].double()
        R = A @ Bc.t()
        tol = 2e-6 * (A.abs() @ Bc.abs().t()) + 1e-30
        err = (C[:, c * sub : (c + 1) * sub] - R).abs()
        assert (err <= tol).all(), (c, float((err / tol).max()))
    with pytest.raises(ValueError):
        linalg.mm_h3(Ap, linalg.h3_planes(Ms.to(device)))
