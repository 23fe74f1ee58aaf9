"""Numerics of every HIP kernel against a plain PyTorch fp32 (or fp64) reference of
the same op.  Runs on an MI355X (marked gpu)."""
import math

import pytest
import torch

from evoxmi import random as rnd
from evoxmi.ops import _ext
from evoxmi.ops.linalg import Operand, gemm

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _require_ext():
    assert _ext.load(), f"evoxmi extension must load on a GPU box: {_ext._ERROR!r}"


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30)).item()


@pytest.mark.parametrize("a_rc,b_rc", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(300, 257, 129), (1000, 1000, 1000), (37, 5, 3)])
def test_gemm_layouts(a_rc, b_rc, M, N, K):
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(K, M, generator=g) if a_rc else torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g) if b_rc else torch.randn(N, K, generator=g)
    ref = gemm(Operand(A, rc=a_rc), Operand(B, rc=b_rc), M, N, K)
    out = gemm(Operand(A.cuda(), rc=a_rc), Operand(B.cuda(), rc=b_rc), M, N, K).cpu()
    assert out.shape == ref.shape
    assert _rel(out, ref) < 1e-5


def test_gemm_asymmetric_identity():
    # A = I with an asymmetric B catches a transposed C-write
    n = 64
    I = torch.eye(n)
    B = torch.arange(n * n, dtype=torch.float32).reshape(n, n)
    out = gemm(Operand(I.cuda()), Operand(B.cuda()), n, n, n).cpu()
    assert torch.equal(out, B.T)


def test_gemm_prologue_epilogue_gather_split():
    g = torch.Generator().manual_seed(0)
    P, d, K = 700, 200, 333
    X = torch.randn(P, d, generator=g)
    idx = torch.randperm(P, generator=g)[:K].to(torch.int32)
    m = torch.randn(d, generator=g)
    w = torch.rand(K, generator=g)
    s = torch.tensor([0.7])
    args = lambda dev: (
        Operand(X.to(dev), rc=True, gather=idx.to(dev), sub=m.to(dev), kw=w.to(dev), sscale=s.to(dev), sscale_inv=True),
        Operand(X.to(dev), rc=True, gather=idx.to(dev), sub=m.to(dev), sscale=s.to(dev), sscale_inv=True),
        d, d, K,
    )
    ref = gemm(*args("cpu"), splits=4)
    out = gemm(*args("cuda"), splits=4).cpu()
    assert out.shape == ref.shape
    assert _rel(out.sum(0), ref.sum(0)) < 1e-5
    # bias + device alpha + k-scale
    Z = torch.randn(50, 40, generator=g)
    Bm = torch.randn(30, 40, generator=g)
    D = torch.rand(40, generator=g)
    bias = torch.randn(30, generator=g)
    al = torch.tensor([2.5])
    r = gemm(Operand(Z, kscale=D), Operand(Bm), 50, 30, 40, alpha_ptr=al, bias_n=bias)
    o = gemm(Operand(Z.cuda(), kscale=D.cuda()), Operand(Bm.cuda()), 50, 30, 40, alpha_ptr=al.cuda(), bias_n=bias.cuda()).cpu()
    assert _rel(o, r) < 1e-5
    assert _rel(r, 2.5 * (Z * D) @ Bm.T + bias) < 1e-5


@pytest.mark.parametrize("n", [1, 7, 1000, 10000, 16384])
def test_argsort(n):
    from evoxmi.ops.sort import argsort

    x = torch.randn(n)
    if n > 10:
        x[3] = x[5]  # tie → index order
        x[7] = float("nan")
    k, i = argsort(x.cuda())
    rk, ri = torch.sort(x, stable=True)
    assert torch.equal(i.cpu(), ri)
    assert torch.allclose(k.cpu(), rk, equal_nan=True)
    k, i = argsort(x.cuda(), descending=True)
    rk, ri = torch.sort(x, descending=True, stable=True)
    assert torch.allclose(k.cpu()[~torch.isnan(rk)], rk[~torch.isnan(rk)])


@pytest.mark.parametrize("n", [2048, 10000, 16384])
def test_lds_bitonic_argsort_kernel(n):
    """The single-workgroup LDS kernel itself (argsort() routes n > 2048 to the library sort)."""
    x = torch.randn(n)
    x[3] = x[5]
    k, i = _ext.ops().argsort_f32(x.cuda(), 0)
    rk, ri = torch.sort(x, stable=True)
    assert torch.equal(i.cpu().long(), ri) and torch.equal(k.cpu(), rk)


@pytest.mark.parametrize("name", ["sphere", "ackley", "rastrigin", "rosenbrock", "griewank", "schwefel", "ellipsoid"])
@pytest.mark.parametrize("d", [2, 30, 1000])
def test_classic_kernels(name, d):
    from evoxmi.problems.numerical import classic

    X = torch.rand(257, d) * 10 - 5
    fn = getattr(classic, f"{name}_func")
    if name == "ackley":
        ref = fn(20.0, 0.2, 2 * math.pi, X.double()).float()
        out = fn(20.0, 0.2, 2 * math.pi, X.cuda()).cpu()
    else:
        ref = fn(X.double()).float()
        out = fn(X.cuda()).cpu()
    assert torch.allclose(out, ref, rtol=2e-4, atol=2e-4)


@pytest.mark.parametrize("fid", list(range(17)))
def test_cec_basic_kernels(fid):
    from evoxmi.problems.numerical import cec2022 as cec

    g = torch.Generator().manual_seed(fid)
    Z = torch.rand(64, 37, generator=g) * 40 - 20
    perm = torch.randperm(37, generator=g).to(torch.int32)
    sub = torch.randn(37, generator=g)
    for args in [dict(), dict(perm=perm, start=5, length=20), dict(sub=sub, scale=0.5)]:
        prob = cec.F1_CEC2022()
        ref = prob._basic(Z.double(), fid, **{k: (v if not isinstance(v, torch.Tensor) or v.dtype != torch.float32 else v.double()) for k, v in args.items()})
        out = prob._basic(Z.cuda(), fid, **{k: (v.cuda() if isinstance(v, torch.Tensor) else v) for k, v in args.items()}).cpu()
        assert torch.allclose(out.double(), ref, rtol=1e-3, atol=1e-3), (fid, args, out[:4], ref[:4])


@pytest.mark.parametrize("f", list(range(1, 13)))
@pytest.mark.parametrize("D", [10, 20, 100])
def test_cec2022_gpu_matches_cpu(f, D):
    from evoxmi.problems.numerical import CEC2022TestSuit

    p = CEC2022TestSuit.create(f)
    X = torch.rand(50, D, generator=torch.Generator().manual_seed(f * D)) * 200 - 100
    ref, _ = p.evaluate(None, X)
    out, _ = p.evaluate(None, X.cuda())
    assert torch.allclose(out.cpu(), ref, rtol=2e-3, atol=1e-3), (f, D, out[:3], ref[:3])


@pytest.mark.parametrize("f", [1, 2, 4])
@pytest.mark.parametrize("rows", [1250, 5000])
def test_cec2022_d1000_shard_rows_match_cpu(f, rows):
    """A population shard of the flagship (λ = 10 000 over 8 / 2 ranks) evaluates its rows on the
    f16x3 rotation with the fused row terms at the shorter tile heights (csrc/kernels/gemm_blk.hip
    evx_gemm_h3): equal to the CPU evaluation; Zakharov (F1) against a float64 evaluation at the
    bound of its conditioning — Σ ½·i·z cancels over 1000 terms of both signs and enters as its
    fourth power, so the f32 CPU result itself is off by up to ~1e-2 on such rows."""
    from evoxmi.ops import linalg
    from evoxmi.problems.numerical import CEC2022TestSuit

    assert linalg.tall_nt_ok(rows, 1000, 1000, torch.device("cuda"))
    p = CEC2022TestSuit.create(f)
    X = torch.rand(rows, 1000, generator=torch.Generator().manual_seed(f + rows)) * 200 - 100
    out, _ = p.evaluate(None, X.cuda())
    out = out.cpu().double()
    if f == 1:
        c = p._consts(1000, torch.device("cpu"))
        z = (X.double() - c["Os"][:1000].double()) @ c["M"].double().t()
        hi = 0.5 * torch.arange(1, 1001, dtype=torch.float64)
        s2, a2 = (hi * z).sum(1), (hi * z).abs().sum(1)
        ref = (z * z).sum(1) + s2 ** 2 + s2 ** 4
        scale = (z * z).sum(1) + a2 ** 2 + a2 ** 4
        cpu, _ = p.evaluate(None, X)
        assert ((cpu.double() - ref).abs() <= 1e-4 * scale).all()  # the reference formula is the suite's
        err = (out - ref).abs() / scale
    else:
        ref, _ = p.evaluate(None, X)
        err = (out - ref.double()).abs() / ref.double().abs()
    assert float(err.max()) <= 1e-4, (f, rows, float(err.max()))


@pytest.mark.parametrize("f", [9, 10, 11, 12])
def test_cec2022_compositions_d1000_fused_path(f):
    """d = 1000 at a population that takes the stacked f16x3 GEMM (one split of X into every
    component's x − o_c planes) and the one-pass composition kernel: equal to the CPU
    evaluation and to the per-component device path; rows at / near a component's optimum
    exercise the zero-distance selection and the weights."""
    from evoxmi import config
    from evoxmi.problems.numerical import CEC2022TestSuit

    p = CEC2022TestSuit.create(f)
    g = torch.Generator().manual_seed(f)
    X = torch.rand(2048, 1000, generator=g) * 200 - 100
    Os = p._consts(1000, torch.device("cpu"))["Os"]
    X[0] = Os[0, :1000]
    X[1] = Os[1, :1000] + 1e-3 * torch.randn(1000, generator=g)
    X[2] = Os[0, :1000] + 1.0
    ref, _ = p.evaluate(None, X)
    out, _ = p.evaluate(None, X.cuda())
    with config.override(cec_compose_fused=0):
        unfused, _ = p.evaluate(None, X.cuda())
    # atol: a row at a Schwefel optimum is Σ of 1000 terms of ±419 cancelling to ~0 (f32
    # summation-order noise ~1e-2 between kernels / the CPU)
    assert torch.allclose(out.cpu(), ref, rtol=2e-3, atol=5e-2), (f, out[:3], ref[:3])
    assert torch.allclose(out.cpu(), unfused.cpu(), rtol=1e-4, atol=5e-2), (f, out[:3], unfused[:3])


@pytest.mark.parametrize("f", [1, 4])
def test_cec2022_rowterms_in_the_h3_epilogue(f):
    """F1 (Zakharov) / F4 (Rastrigin) at d = 1000 on the f16x3 rotation with the row terms reduced
    in the GEMM epilogue (transposing butterfly over each 32-column block, the 128-column tiles
    summed in order): equal to the CPU evaluation and to GEMM + basic-function kernel; rows at
    the optimum give 0 (the < 1e-8 clamp)."""
    from evoxmi import config
    from evoxmi.problems.numerical import CEC2022TestSuit

    p = CEC2022TestSuit.create(f)
    g = torch.Generator().manual_seed(40 + f)
    X = torch.rand(2050, 1000, generator=g) * 200 - 100
    Os = p._consts(1000, torch.device("cpu"))["Os"]
    o = (Os if Os.dim() == 1 else Os[0])[:1000]
    X[0] = o
    X[1] = o + 1e-2 * torch.randn(1000, generator=g)
    ref, _ = p.evaluate(None, X)
    out, _ = p.evaluate(None, X.cuda())
    with config.override(cec_rowterms_h3=0):
        plain, _ = p.evaluate(None, X.cuda())
    assert float(out[0]) == 0.0
    if f == 1:
        # fp64 reference with an error bound: b = Σ ½(j+1) z is a cancelling sum, and b⁴
        # amplifies its absolute error δb ≤ ε·Σ|½(j+1) z| by 4|b|³
        M = p._consts(1000, torch.device("cpu"))["M"].double()
        Z = (X.double() - o.double()) @ M.t()
        c = 0.5 * torch.arange(1, 1001, dtype=torch.float64)
        b = Z @ c
        R = (Z * Z).sum(1) + b**2 + b**4
        db = 1e-5 * (Z.abs() @ c)
        tol = 1e-5 * (Z * Z).sum(1) + (2 * b.abs() + 4 * b.abs() ** 3) * db + 4 * db**4 + 1e-3
        for got in (out.cpu().double(), plain.cpu().double()):
            assert ((got - R).abs() <= tol).all(), float(((got - R).abs() / tol).max())
    else:
        assert torch.allclose(out.cpu(), ref, rtol=1e-4, atol=1e-2), (f, out[:3], ref[:3])
        assert torch.allclose(out.cpu(), plain.cpu(), rtol=1e-4, atol=1e-2)


def test_pso_kernel_matches_cpu():
    from evoxmi.ops.pso import pso_update

    g = torch.Generator().manual_seed(3)
    n, d = 100, 13
    pop, vel, lbl = torch.randn(n, d, generator=g), torch.randn(n, d, generator=g), torch.randn(n, d, generator=g)
    lbf, fit = torch.randn(n, generator=g), torch.randn(n, generator=g)
    gbl = torch.randn(d, generator=g)
    lb, ub = -torch.ones(d) * 2, torch.ones(d) * 2
    kp, kg = rnd.split(rnd.PRNGKey(5))
    ref = pso_update(pop, vel, lbl, lbf, fit, gbl, kp, kg, 0.6, 2.5, 0.8, lb, ub)
    cu = lambda t: t.cuda()
    out = pso_update(*map(cu, (pop, vel, lbl, lbf, fit, gbl, kp, kg)), 0.6, 2.5, 0.8, cu(lb), cu(ub))
    for a, b in zip(out, ref):
        assert torch.allclose(a.cpu(), b, atol=1e-5)


def test_cmaes_gpu_converges_sphere():
    from evoxmi.algorithms import CMAES
    from evoxmi.monitors import EvalMonitor
    from evoxmi.problems.numerical import Sphere
    from evoxmi.workflows import StdWorkflow

    alg = CMAES(torch.tensor([5.0, -10, 15, -20, 25], device="cuda"), init_stdev=0.1, pop_size=10)
    mon = EvalMonitor()
    wf = StdWorkflow(alg, Sphere(), monitors=[mon])
    st = wf.init(rnd.PRNGKey(42, device="cuda"))
    for _ in range(200):
        st = wf.step(st)
    assert mon.get_best_fitness().item() < 0.1


def test_cmaes_graph_mode_matches_eager():
    from evoxmi.algorithms import CMAES
    from evoxmi.problems.numerical import F1_CEC2022
    from evoxmi.workflows import StdWorkflow

    d = 64
    outs = []
    for graph in (False, True):
        alg = CMAES(torch.zeros(d, device="cuda"), init_stdev=10.0, pop_size=256)
        wf = StdWorkflow(alg, F1_CEC2022(), graph=graph)
        st = wf.init(rnd.PRNGKey(7, device="cuda"))
        for _ in range(6):
            st = wf.step(st)
        outs.append(st.get_child_state("algorithm").mean.clone())
    assert torch.allclose(outs[0], outs[1], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("n", [5, 30, 100, 257, 1000])
def test_jacobi_cold_eigh(n):
    from evoxmi.ops import jacobi

    g = torch.Generator().manual_seed(n)
    X = torch.randn(n, n, generator=g, dtype=torch.float64)
    C = (X @ X.T / n + torch.eye(n, dtype=torch.float64)).float()
    w, V = jacobi.eigh(C.cuda())
    w, V = w.cpu().double(), V.cpu().double()
    Cd = C.double()
    rec = (V * w) @ V.T
    assert ((rec - Cd).norm() / Cd.norm()).item() < 3e-5 * max(1, n / 100) ** 0.5
    assert ((V.T @ V - torch.eye(n, dtype=torch.float64)).norm() / math.sqrt(n)).item() < 2e-5
    wr = torch.linalg.eigvalsh(Cd)
    assert torch.allclose(w, wr, rtol=1e-4, atol=1e-4 * wr.abs().max().item())


@pytest.mark.parametrize("n,sweeps", [(100, 3), (1000, 2), (300, 1), (16, 2), (3990, 1)])
def test_jacobi_fused_apply_solve_is_bit_identical(n, sweeps):
    """The fused launch (round t's apply + round t+1's solves, cross-workgroup counters)
    computes exactly the same rotations as separate solve/apply launches."""
    from evoxmi import config
    from evoxmi.ops import jacobi

    g = torch.Generator().manual_seed(n)
    Q, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    lam = 1 + 0.05 * torch.rand(n, generator=g, dtype=torch.float64)
    X = torch.randn(n, n, generator=g, dtype=torch.float64) * 1e-2
    C = ((Q * lam) @ Q.T + (X + X.T)).float().cuda()
    outs = []
    for fused in (0, 1, 2):  # split launches / fused apply+solve / B update inside the next solve launch
        outs.append(jacobi.warm_eigh(C, Q.float().cuda(), max_sweeps=sweeps, fused=fused))
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1])


def test_jacobi_warm_start_converges_fast():
    from evoxmi.ops import jacobi

    n = 1000
    g = torch.Generator().manual_seed(0)
    Q, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    lam = torch.logspace(0, 3, n, dtype=torch.float64)
    C0 = (Q * lam) @ Q.T
    Y = torch.randn(2000, n, generator=g, dtype=torch.float64) @ (Q * lam.sqrt()).T
    C1 = 0.995 * C0 + 0.005 * (Y.T @ Y) / 2000
    w, B, stats = jacobi.warm_eigh(C1.float().cuda(), Q.float().cuda(), return_stats=True)
    w, B = w.cpu().double(), B.cpu().double()
    rec = (B * w) @ B.T
    assert ((rec - C1).norm() / C1.norm()).item() < 3e-5
    assert ((B.T @ B - torch.eye(n, dtype=torch.float64)).norm() / math.sqrt(n)).item() < 3e-5


def test_jacobi_warm_chain_stays_orthonormal():
    """CMA-ES-like chain: a clustered spectrum (eigenvalues within ±5 % of 1) nudged by a
    rank-μ term every step.  The converged solver (Jacobi hand-off + sorted-block
    refinement, evoxmi/ops/sbr.py) must reach the tolerance at every step and the carried
    basis must stay orthonormal."""
    from evoxmi.ops import sbr

    n = 500
    g = torch.Generator(device="cuda").manual_seed(3)
    C = torch.eye(n, device="cuda")
    B = torch.eye(n, device="cuda")
    eye = torch.eye(n, device="cuda", dtype=torch.float64)
    for _ in range(40):
        Y = torch.randn(1000, n, device="cuda", generator=g)
        C = 0.99 * C + 0.01 * (Y.T @ Y) / 1000
        w, B, info = sbr.eigh_warm(C, B)
        assert info.off_rel <= 1e-5, info
        res = ((B.double() * w.double()) @ B.double().T - C.double()).norm() / C.double().norm()
        assert res.item() < 2e-5
    orth = (B.double().T @ B.double() - eye).norm().item()
    assert orth < 1e-4


@pytest.mark.parametrize("n,type", [(64, 1), (63, 1), (64, 2), (4096, 1)])
def test_sbx_kernel_matches_cpu(n, type):
    from evoxmi.operators.crossover import simulated_binary

    x = torch.rand(n, 37, generator=torch.Generator().manual_seed(n))
    key = rnd.PRNGKey(11)
    ref = simulated_binary(key, x, 0.9, 20.0, type)
    out = simulated_binary(key.cuda(), x.cuda(), 0.9, 20.0, type).cpu()
    assert out.shape == ref.shape
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("n", [2, 63, 1000])
def test_pm_kernel_matches_cpu(n):
    from evoxmi.operators.mutation import polynomial

    x = torch.rand(n, 29, generator=torch.Generator().manual_seed(n)) * 4 - 2
    lb, ub = -torch.ones(29), torch.ones(29)
    key = rnd.PRNGKey(5)
    ref = polynomial(key, x, (lb, ub), 5.0, 20.0)
    out = polynomial(key.cuda(), x.cuda(), (lb.cuda(), ub.cuda()), 5.0, 20.0).cpu()
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("n,m", [(1, 2), (100, 2), (1000, 3), (8192, 3), (300, 5)])
def test_nds_kernel_matches_cpu(n, m):
    from evoxmi.operators.selection import non_dominated_sort

    f = torch.rand(n, m, generator=torch.Generator().manual_seed(n))
    if n > 10:
        f[5] = f[3]  # duplicates are mutually non-dominated
    ref = non_dominated_sort(f)
    out = non_dominated_sort(f.cuda()).cpu()
    assert torch.equal(out.to(torch.int32), ref.to(torch.int32))


@pytest.mark.parametrize("n,m,until", [(8192, 3, 4097), (2000, 2, 700), (700, 4, 1)])
def test_nds_kernel_until(n, m, until):
    """Peeling stops once >= `until` rows are ranked: those ranks are exact, the rest get n."""
    from evoxmi.operators.selection import non_dominated_sort

    f = torch.rand(n, m, generator=torch.Generator().manual_seed(n + m))
    ref = non_dominated_sort(f).to(torch.int32)
    out = non_dominated_sort(f.cuda(), until=until).cpu()
    cut = int(torch.sort(ref).values[until - 1])
    exact = ref <= cut
    assert torch.equal(out[exact], ref[exact])
    assert (out[~exact] == n).all()


def test_nds_under_graph_capture():
    from evoxmi.operators.selection import non_dominated_sort

    x = torch.rand(3000, 3, device="cuda")
    out = torch.empty(3000, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        non_dominated_sort(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out.copy_(non_dominated_sort(x))
    for seed in range(3):
        x.copy_(torch.rand(3000, 3, generator=torch.Generator().manual_seed(seed)).cuda())
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out.cpu(), non_dominated_sort(x.cpu()).to(torch.int32))


def test_crowding_gpu_matches_cpu():
    from evoxmi.operators.selection import crowding_distance

    f = torch.rand(500, 3, generator=torch.Generator().manual_seed(1))
    mask = torch.rand(500, generator=torch.Generator().manual_seed(2)) < 0.4
    ref = crowding_distance(f, mask)
    out = crowding_distance(f.cuda(), mask.cuda()).cpu()
    fin = torch.isfinite(ref)
    assert torch.equal(fin, torch.isfinite(out))
    assert torch.allclose(out[fin], ref[fin], rtol=1e-5, atol=1e-6)
    assert torch.equal(out[~fin], ref[~fin])


@pytest.mark.parametrize("variant", [1, 2, 3, 4])
@pytest.mark.parametrize("n,d,m", [(7, 7, 3), (1000, 12, 3), (333, 100, 10)])
def test_dtlz_fused_kernel(variant, n, d, m):
    from evoxmi.problems.numerical import DTLZ1, DTLZ2, DTLZ3, DTLZ4

    cls = {1: DTLZ1, 2: DTLZ2, 3: DTLZ3, 4: DTLZ4}[variant]
    p = cls(d=d, m=m)
    X = torch.rand(n, d, generator=torch.Generator().manual_seed(n + variant))
    ref, _ = p.evaluate(None, X)
    out, _ = p.evaluate(None, X.cuda())
    assert torch.allclose(out.cpu(), ref, rtol=2e-4, atol=1e-4)


def test_maf_on_gpu_matches_cpu():
    from evoxmi.problems.numerical import maf

    X = torch.rand(64, 12, generator=torch.Generator().manual_seed(3))
    for i in range(1, 16):
        p = getattr(maf, f"MaF{i}")(d=12, m=3)
        ref, _ = p.evaluate(None, X)
        out, _ = p.evaluate(None, X.cuda())
        assert torch.allclose(out.cpu(), ref, rtol=1e-4, atol=1e-4), i


@pytest.mark.parametrize("R,d,K", [(1, 1, 1), (100, 20, 6), (3000, 257, 9), (64, 1000, 16)])
def test_de_trial_kernel(R, d, K):
    from evoxmi.ops.evo import de_trial

    g = torch.Generator().manual_seed(R + d)
    rows = 2 * R + 3
    P = torch.randn(rows, d, generator=g) * 50
    idx = torch.randint(0, rows, (R, K), generator=g)
    coef = torch.randn(R, K, generator=g)
    coef[coef.abs() < 0.3] = 0
    cur = torch.randint(0, rows, (R,), generator=g)
    mode = torch.randint(0, 3, (R,), generator=g)
    CR = torch.rand(R, generator=g)
    jr = torch.randint(0, d, (R,), generator=g)
    L = torch.randint(0, d, (R,), generator=g)
    lb, ub = torch.full((d,), -60.0), torch.full((d,), 60.0)
    key = rnd.PRNGKey(R)
    for rep in ("clip", "midpoint", "none"):
        ref = de_trial(key, P, idx, coef, cur, mode, CR, jr, L, lb, ub, rep)
        c = lambda t: t.cuda()
        out = de_trial(c(key), c(P), c(idx), c(coef), c(cur), c(mode), c(CR), c(jr), c(L), c(lb), c(ub), rep).cpu()
        assert torch.allclose(out, ref, rtol=1e-5, atol=1e-3), rep


@pytest.mark.parametrize("name", ["DE", "ODE", "CoDE", "JaDE", "SaDE", "SHADE", "LSHADE", "ILSHADE", "JSO", "LSHADE_RSP", "EPSDE", "EVDE"])
def test_de_variants_graph_matches_eager(name):
    """A DE generation captured in a hipGraph replays to the same state as eager."""
    from evoxmi.algorithms import de_variants as dv
    from evoxmi.problems.numerical import CEC2022TestSuit
    from evoxmi.workflows import StdWorkflow

    D = 10
    lb, ub = torch.full((D,), -100.0, device="cuda"), torch.full((D,), 100.0, device="cuda")
    outs = []
    for graph in (False, True):
        algo = getattr(dv, name)(lb=lb, ub=ub, pop_size=100)
        wf = StdWorkflow(algo, CEC2022TestSuit.create(1), graph=graph)
        st = wf.init(rnd.PRNGKey(7, device="cuda"))
        for i in range(6):
            st = wf.step(st)
            a = st.get_child_state("algorithm")
            if "progress" in a.keys():
                st = st.update_child("algorithm", a.update(progress=(i + 1) / 10))
        outs.append(st.get_child_state("algorithm").fitness.clone())
    fin = torch.isfinite(outs[0])
    assert torch.equal(fin, torch.isfinite(outs[1]))
    assert torch.allclose(outs[0][fin], outs[1][fin], rtol=1e-5, atol=1e-4)


def test_topk_safe_under_graph_capture():
    """ops.sort.topk replayed from a hipGraph matches torch.topk on the CPU."""
    from evoxmi.ops.sort import topk

    x = torch.randn(500, 3000, device="cuda")
    out_i = torch.empty((500, 3), dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        topk(x, 3)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out_i.copy_(topk(x, 3)[1])
    for seed in range(3):
        x.copy_(torch.randn(500, 3000, generator=torch.Generator().manual_seed(seed)).cuda())
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out_i.cpu(), torch.topk(x.cpu(), 3).indices)


ES_GRAPH = ["CSO", "CLPSO", "SLPSOGS", "DMSPSOEL", "FIPS", "SwmmPSO", "FSPSO", "OpenES", "PGPE", "SNES", "DES", "ARS", "ESMC", "CR_FM_NES", "PersistentES", "NoiseReuseES", "SeparableNES",
            "MAES", "LMMAES", "RMES", "AMaLGaM", "IndependentAMaLGaM", "SepCMAES", "LES"]


@pytest.mark.parametrize("name", ES_GRAPH)
def test_es_variants_graph_matches_eager(name):
    import evoxmi.algorithms as A
    from evoxmi.problems.numerical import Sphere
    from evoxmi.workflows import StdWorkflow
    import warnings

    mean = torch.tensor([5.0, -10, 15, -20, 25, 1, 2, 3], device="cuda")
    lb, ub = torch.full((8,), -32.0, device="cuda"), torch.full((8,), 32.0, device="cuda")
    mk = {
        "CSO": lambda: A.CSO(lb, ub, 64), "SLPSOGS": lambda: A.SLPSOGS(lb, ub, 64, 0.01, 0.7),
        "CLPSO": lambda: A.CLPSO(lb, ub, 64, 0.5, 1.5, torch.full((64,), 0.05, device="cuda")),
        "DMSPSOEL": lambda: A.DMSPSOEL(lb, ub, 3, 9, 37, 3, 5, 0.7, 1.5, 1.5, 1.5, 1.5), "FIPS": lambda: A.FIPS(lb, ub, 64),
        "SwmmPSO": lambda: A.SwmmPSO(lb, ub, 64), "FSPSO": lambda: A.FSPSO(lb, ub, 64),
        "OpenES": lambda: A.OpenES(mean, 64, learning_rate=1, noise_stdev=3, optimizer="adam"),
        "PGPE": lambda: A.PGPE(64, mean, optimizer="clipup", stdev_init=3.0),
        "SNES": lambda: A.SNES(64, mean, sigma=3.0), "DES": lambda: A.DES(64, mean, sigma_init=3.0),
        "ARS": lambda: A.ARS(64, mean, lr=0.5, sigma=1.0), "ESMC": lambda: A.ESMC(65, mean, lr=0.5, sigma=1.0),
        "CR_FM_NES": lambda: A.CR_FM_NES(64, mean, sigma=3.0), "PersistentES": lambda: A.PersistentES(64, mean, lr=0.5),
        "NoiseReuseES": lambda: A.NoiseReuseES(64, mean, lr=0.5),
        "SeparableNES": lambda: A.SeparableNES(mean, torch.ones(8, device="cuda") * 3, pop_size=64),
        "MAES": lambda: A.MAES(mean, init_stdev=1.0, pop_size=20), "LMMAES": lambda: A.LMMAES(mean, init_stdev=1.0, pop_size=20),
        "RMES": lambda: A.RMES(mean, init_stdev=1.0, pop_size=20), "AMaLGaM": lambda: A.AMaLGaM(mean, init_stdev=1.0, pop_size=20),
        "IndependentAMaLGaM": lambda: A.IndependentAMaLGaM(mean, init_stdev=1.0, pop_size=20),
        "SepCMAES": lambda: A.SepCMAES(mean, init_stdev=1.0, pop_size=20), "LES": lambda: A.LES(64, mean, sigma_init=3.0),
    }[name]
    outs = []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for graph in (False, True):
            wf = StdWorkflow(mk(), Sphere(), graph=graph)
            st = wf.init(rnd.PRNGKey(3, device="cuda"))
            for _ in range(6):
                st = wf.step(st)
            a = st.get_child_state("algorithm")
            k = next(k for k in ("center", "mean", "population") if k in a.keys())
            outs.append(a[k].clone())
    assert torch.allclose(outs[0], outs[1], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("func", ["tchebycheff", "pbi", "weighted_sum", "modified_tchebycheff"])
@pytest.mark.parametrize("nr,update_z", [(2, True), (64, False)])
def test_moead_scan_kernel(func, nr, update_z):
    from evoxmi.ops.mo import moead_scan

    g = torch.Generator().manual_seed(7)
    N, R, T, M = 300, 300, 30, 3
    objs, off = torch.rand(N, M, generator=g), torch.rand(R, M, generator=g) * 0.9
    P = torch.randint(0, N, (R, T), generator=g)
    W = torch.rand(N, M, generator=g) + 0.05
    z = torch.zeros(M) - 0.01
    ref = moead_scan(objs, off, P, W, z, func, nr=nr, update_z=update_z)
    out = moead_scan(objs.cuda(), off.cuda(), P.cuda(), W.cuda(), z.cuda(), func, nr=nr, update_z=update_z)
    assert torch.equal(out[0].cpu(), ref[0])
    assert torch.allclose(out[1].cpu(), ref[1]) and torch.allclose(out[2].cpu(), ref[2])


@pytest.mark.parametrize("name", ["NSGA2", "NSGA3", "MOEAD", "MOEADDRA", "EAGMOEAD", "RVEA", "IBEA", "HypE", "SPEA2", "TDEA", "LMOCSO"])
def test_moea_on_gpu(name):
    import evoxmi.algorithms as A
    from evoxmi.problems.numerical import DTLZ2
    from evoxmi.workflows import StdWorkflow

    lb, ub = torch.zeros(12, device="cuda"), torch.ones(12, device="cuda")
    algo = getattr(A, name)(3, lb, ub, 100) if name == "LMOCSO" else getattr(A, name)(lb, ub, 3, 100)
    wf = StdWorkflow(algo, DTLZ2(d=12, m=3))
    st = wf.init(rnd.PRNGKey(1, device="cuda"))
    for _ in range(5):
        st = wf.step(st)
    f = st.get_child_state("algorithm").fitness
    assert f.is_cuda and torch.isfinite(f[~torch.isnan(f).any(1)]).all()


@pytest.mark.parametrize("cap,hidden", [(1, 64), (5, 64), (20, 64), (20, 40), (20, 96)])
def test_ant_rollout_kernel_matches_torch(cap, hidden):
    """Fused LDS-resident Ant rollout vs the torch reference env + batched MLP."""
    from evoxmi.models import MLPPolicy
    from evoxmi.problems.neuroevolution import Brax
    from evoxmi.utils import TreeAndVector

    policy = MLPPolicy([27, hidden, hidden, 8])
    params = policy.init(rnd.PRNGKey(0))
    tv = TreeAndVector(params)
    pop = tv.to_vector(params) + 0.3 * torch.randn(96, tv.to_vector(params).numel(), generator=torch.Generator().manual_seed(cap))
    tree = tv.batched_to_tree(pop)
    ref, _ = Brax(policy, "ant", cap, fused=False).evaluate(Brax(policy, "ant", cap).init(rnd.PRNGKey(5)), tree)
    tree_g = torch.utils._pytree.tree_map(lambda x: x.cuda(), tree)
    prob = Brax(policy, "ant", cap)
    out, _ = prob.evaluate(prob.init(rnd.PRNGKey(5)), tree_g)
    assert prob._fused_ok(tree_g)
    assert torch.allclose(out.cpu(), ref, rtol=2e-3, atol=2e-3 * cap)


def test_ant_rollout_long_episode_statistics():
    from evoxmi.models import MLPPolicy
    from evoxmi.problems.neuroevolution import Brax
    from evoxmi.utils import TreeAndVector

    policy = MLPPolicy([27, 32, 32, 8])
    params = policy.init(rnd.PRNGKey(1))
    tv = TreeAndVector(params)
    pop = tv.to_vector(params) + 0.2 * torch.randn(256, tv.to_vector(params).numel(), generator=torch.Generator().manual_seed(0))
    tree = tv.batched_to_tree(pop)
    ref, _ = Brax(policy, "ant", 300, fused=False).evaluate(Brax(policy, "ant", 300).init(rnd.PRNGKey(2)), tree)
    prob = Brax(policy, "ant", 300)
    out, _ = prob.evaluate(prob.init(rnd.PRNGKey(2)), torch.utils._pytree.tree_map(lambda x: x.cuda(), tree))
    # chaotic dynamics: individual returns may diverge late in the episode, the population statistics must not
    assert abs(float(out.mean()) - float(ref.mean())) < 0.05 * float(ref.abs().mean()) + 1.0
    assert torch.isfinite(out).all()


# ---------------------------------------------------------------- MOEA/D generation kernels
def test_moead_parents_matches_argsort():
    from evoxmi.ops.mo import moead_parents

    N, T = 300, 77
    nb = torch.randint(0, N, (N, T), generator=torch.Generator().manual_seed(0))
    key = rnd.PRNGKey(9)
    perm = torch.argsort(rnd.uniform(key, (N, T)), dim=1, stable=True)[:, :2]
    ref = torch.gather(nb, 1, perm)
    p0, p1 = moead_parents(nb.cuda(), key.cuda())
    assert torch.equal(p0.cpu().long(), ref[:, 0]) and torch.equal(p1.cpu().long(), ref[:, 1])


@pytest.mark.parametrize("d", [64, 37])
def test_moead_variation_matches_operators(d):
    from evoxmi.operators.crossover import SimulatedBinary
    from evoxmi.operators.mutation import Polynomial
    from evoxmi.ops.mo import moead_variation

    N = 101
    g = torch.Generator().manual_seed(d)
    pop = torch.rand(N, d, generator=g) * 4 - 2
    lb, ub = torch.full((d,), -2.0), torch.full((d,), 2.0)
    p0, p1 = torch.randint(0, N, (N,), generator=g), torch.randint(0, N, (N,), generator=g)
    kx, km = rnd.PRNGKey(1), rnd.PRNGKey(2)
    off = SimulatedBinary(type=2)(kx, torch.cat([pop[p0], pop[p1]], 0))
    ref = torch.clamp(Polynomial((lb, ub))(km, off), lb, ub)
    c = lambda t: t.cuda()
    out = moead_variation(c(pop), c(p0).int(), c(p1).int(), c(kx), c(km), c(lb), c(ub), 1.0, 20.0, 1.0, 20.0).cpu()
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("func", ["tchebycheff", "pbi", "weighted_sum", "modified_tchebycheff", "tchebycheff_norm"])
def test_moead_replace_matches_sequential(func):
    from evoxmi.algorithms.mo.moead import moead_replace, moead_replace_sequential, reverse_neighbors
    from evoxmi.ops import mo as mo_ops
    from evoxmi.utils.common import AggregationFunction

    N, T, M, d = 200, 20, 3, 5
    g = torch.Generator().manual_seed(3)
    w = torch.rand(N, M, generator=g) + 0.05
    nb = torch.argsort(torch.rand(N, N, generator=g), 1)[:, :T]
    pop_obj, off_obj = torch.rand(N, M, generator=g), torch.rand(N, M, generator=g)
    pop, off = torch.rand(N, d, generator=g), torch.rand(N, d, generator=g)
    z, zmax = torch.zeros(M) - 0.01, torch.ones(M) * 1.1
    agg = AggregationFunction(func)
    ref_pop, ref_obj = moead_replace_sequential(pop, pop_obj, off, off_obj, w, z, zmax, nb, agg)
    rowptr, _, owner = reverse_neighbors(nb.cuda())
    c = lambda t: t.cuda()
    win, new_obj = mo_ops.moead_replace(c(pop_obj), c(off_obj), c(w), c(z), c(zmax), rowptr.int(), owner.int(), func)
    new_pop = mo_ops.moead_select_rows(c(pop), c(off), win)
    assert torch.allclose(new_obj.cpu(), ref_obj) and torch.allclose(new_pop.cpu(), ref_pop)


@pytest.mark.parametrize("cls", ["LSMOP1", "LSMOP2", "LSMOP3", "LSMOP4", "LSMOP5", "LSMOP6", "LSMOP7", "LSMOP8", "LSMOP9"])
def test_lsmop_fused_matches_eager(cls):
    import evoxmi.problems.numerical as P

    prob = getattr(P, cls)(d=300, m=3)
    X = torch.rand(64, 300, generator=torch.Generator().manual_seed(4))
    ub = torch.cat([torch.ones(2), 10 * torch.ones(298)])
    X = X * ub
    ref, _ = prob.evaluate(None, X)
    out, _ = prob.evaluate(None, X.cuda())
    assert torch.allclose(out.cpu(), ref, rtol=2e-4, atol=1e-3)


def test_openes_ant_graph_matches_eager():
    """A whole OpenES + fused Ant-rollout generation replays from a hipGraph."""
    from evoxmi.algorithms import OpenES
    from evoxmi.models import MLPPolicy
    from evoxmi.problems.neuroevolution import Brax
    from evoxmi.utils import TreeAndVector, rank_based_fitness
    from evoxmi.workflows import StdWorkflow

    outs = []
    for graph in (False, True):
        policy = MLPPolicy([27, 32, 32, 8])
        params = policy.init(rnd.PRNGKey(1), device="cuda")
        tv = TreeAndVector(params)
        wf = StdWorkflow(OpenES(tv.to_vector(params), 64, learning_rate=0.05, noise_stdev=0.1, optimizer="adam"), Brax(policy, "ant", 80),
                         sol_transforms=[tv.batched_to_tree], fit_transforms=[rank_based_fitness], opt_direction="max", graph=graph)
        st = wf.init(rnd.PRNGKey(3, device="cuda"))
        for _ in range(4):
            st = wf.step(st)
        assert (wf._graph is not None) == graph
        outs.append(st.get_child_state("algorithm").center.clone())
    assert torch.allclose(outs[0], outs[1], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("d", [37, 100, 300])
def test_cmaes_fused_epilogue_matches_torch_ops(d):
    """cmaes.hip epilogue (δ-GEMV, paths, covariance blend + padding, eigenbasis extraction)
    against the reference-shaped torch implementation on the SAME tell inputs.  The eigen-
    basis of a clustered spectrum is ill-conditioned (rounding-level differences in C
    rotate it), so B/D are checked through C ≈ B D² Bᵀ and invsqrtC·C·invsqrtC ≈ I."""
    from evoxmi import config
    from evoxmi.algorithms import CMAES
    from evoxmi.problems.numerical import Rastrigin
    from evoxmi.workflows import StdWorkflow

    alg = CMAES(torch.full((d,), 2.0, device="cuda"), init_stdev=1.5, pop_size=4 * d)
    wf = StdWorkflow(alg, Rastrigin())
    st = wf.init(rnd.PRNGKey(11, device="cuda"))
    for _ in range(3):
        st = wf.step(st)
    a = st.get_child_state("algorithm")
    g = torch.Generator(device="cuda").manual_seed(d)
    dm = 0.1 * torch.randn(d, device="cuda", generator=g)
    Y = torch.randn(alg.mu, d, device="cuda", generator=g)
    S = (Y.T * alg.weights) @ Y
    outs = []
    for fused in (0, 1):
        with config.override(cma_fused=fused):
            outs.append(alg._finish_tell(a, dm, S))
    r, f = outs
    for k in ("mean", "sigma", "ps", "pc"):
        assert torch.allclose(f[k], r[k], rtol=1e-5, atol=1e-6), k
    assert torch.allclose(f.C, r.C, rtol=1e-5, atol=1e-6)
    Cd = 0.5 * (f.C.double() + f.C.double().T)
    eye = torch.eye(d, device="cuda", dtype=torch.float64)

    def quality(o):  # (reconstruction residual, whitening residual) of one decomposition
        rec = (o.B.double() * o.D.double() ** 2) @ o.B.double().T
        W = o.invsqrtC.double()
        return ((rec - Cd).norm() / Cd.norm()).item(), ((W @ Cd @ W - eye).norm() / d**0.5).item()

    (rf, wf_), (rr, wr) = quality(f), quality(r)
    assert rf <= 1.5 * rr + 1e-4 and wf_ <= 1.5 * wr + 1e-4, (rf, rr, wf_, wr)
    assert torch.allclose(torch.sort(f.D).values, torch.sort(r.D).values, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("n,m,N,shift,front", [(8192, 3, 4096, 0, "rand"), (8192, 3, 4096, -1, "rand"), (300, 2, 150, 0, "rand"),
                                                (200, 4, 100, -1, "rand"), (64, 3, 63, 0, "rand"), (8192, 3, 4096, 0, "pareto"),
                                                (3000, 3, 1500, -1, "pareto"), (1500, 2, 750, 0, "pareto")])
def test_nsga_select_kernel_matches_torch(n, m, N, shift, front):
    """Fused NSGA-II selection == non_dominated_sort → crowding on the front of
    sorted(rank)[mask_pos] → lexsort((−cd, rank))[:N] (CPU reference ops).  "pareto"
    puts most rows on one front (the 2/4/8-items-per-thread crowding sorts)."""
    from evoxmi.operators.selection.non_dominate import crowding_distance, lexsort, non_dominated_sort
    from evoxmi.ops.nds import nsga2_survivors

    g = torch.Generator().manual_seed(n + m)
    f = torch.rand(n, m, generator=g)
    if front == "pareto":
        f[n // 8:] = f[n // 8:] / f[n // 8:].sum(1, keepdim=True)  # simplex: mutually non-dominated
    f[: n // 10] = torch.round(f[: n // 10] * 8) / 8  # ties in objective values
    f[5] = f[7]  # duplicate rows
    f[9:12, 0] = torch.tensor([-0.0, 0.0, -0.0])  # signed zeros compare equal (radix keys canonicalised)
    mask_pos = N + shift
    rank = non_dominated_sort(f)
    worst = torch.sort(rank).values[mask_pos]
    cd = crowding_distance(f, rank == worst)
    ref = lexsort([-cd, rank.to(cd.dtype)])[:N]
    out = nsga2_survivors(f.cuda(), N, mask_pos, until=mask_pos + 1).cpu()
    assert torch.equal(out, ref)


def test_nds_barrier_timeout_is_reported():
    """A persistent-peel grid barrier that times out must not return ranks silently: the
    unranked rows go last (rank n) and the sticky kernel error word raises at the next
    check (fault injected with EVOXMI_NDS_FAULT_TEST in a subprocess)."""
    import os
    import subprocess
    import sys

    code = (
        "import torch\n"
        "from evoxmi.ops import _ext, nds\n"
        "f = torch.rand(3000, 3, device='cuda')\n"
        "r = nds.non_dominated_sort(f)\n"
        "torch.cuda.synchronize()\n"
        "assert int(r.min()) >= 0, 'unranked rows must not get rank -1'\n"
        "try:\n"
        "    _ext.check_kernel_errors()\n"
        "except RuntimeError as e:\n"
        "    assert 'nds' in str(e); print('RAISED')\n"
    )
    env = dict(os.environ, EVOXMI_NDS_FAULT_TEST="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "RAISED" in out.stdout


# ---------------------------------------------------------------- K17 / K18 (mo_geom.hip)
@pytest.mark.gpu
@pytest.mark.parametrize("N,M,m,T", [(1000, 1000, 3, 20), (300, 5000, 10, 1), (257, 64, 64, 32), (50, 40, 2, 7)])
def test_knn_kernel_matches_direct_form(N, M, m, T):
    from evoxmi.ops import geom

    g = torch.Generator().manual_seed(N + M)
    X, Y = torch.rand(N, m, generator=g), torch.rand(M, m, generator=g)
    d_ref, i_ref = geom.knn(X, Y, T)
    d, i = geom.knn(X.cuda(), Y.cuda(), T)
    assert torch.allclose(d.cpu(), d_ref, rtol=1e-5, atol=1e-6)
    agree = (i.cpu() == i_ref).float().mean().item()
    assert agree > 0.999, agree  # index order may differ only at rounding-level ties
    # the returned indices are the claimed distances
    dd = torch.sqrt(((X[:, None, :] - Y[i.cpu()]) ** 2).sum(-1))
    assert torch.allclose(dd, d.cpu(), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_knn_kernel_ties_by_index():
    from evoxmi.ops import geom

    # uniform weights on a simplex lattice: many exactly equal distances
    from evoxmi.operators.sampling import UniformSampling

    w = UniformSampling(300, 3)()[0].float()
    d_ref, i_ref = geom.knn(w, w, 20)
    d, i = geom.knn(w.cuda(), w.cuda(), 20)
    assert torch.equal(i.cpu(), i_ref)
    assert torch.allclose(d.cpu(), d_ref, atol=1e-6)


@pytest.mark.gpu
def test_knn_kernel_nan_and_inf_rows():
    from evoxmi.ops import geom

    g = torch.Generator().manual_seed(5)
    X, Y = torch.rand(300, 3, generator=g), torch.rand(40, 3, generator=g)
    X[3, 1] = float("nan")       # every distance of row 3 is NaN
    X[4, 0] = float("inf")       # every distance of row 4 is inf
    Y[7, 2] = float("nan")       # candidate 7 is NaN for every row
    for T in (1, 5):
        d_ref, i_ref = geom.knn(X, Y, T)
        d, i = geom.knn(X.cuda(), Y.cuda(), T)
        assert torch.equal(i.cpu(), i_ref)
        assert torch.allclose(d.cpu(), d_ref, equal_nan=True)
    md = geom.min_dist(X.cuda(), Y.cuda()).cpu()
    ref = torch.cdist(X.double(), Y.double()).min(1).values.float()
    assert torch.isnan(md).all() and torch.isnan(ref).all()  # candidate 7 poisons every row
    md = geom.min_dist(X[:, :2].cuda(), Y[:, :2].cuda()).cpu()
    # direct-form distances (torch.cdist's matmul form turns an inf coordinate into NaN)
    ref = (((X[:, None, :2].double() - Y[None, :, :2].double()) ** 2).sum(-1)).sqrt().min(1).values.float()
    assert torch.isnan(md[3]) and torch.isinf(md[4]) and torch.allclose(md, ref, equal_nan=True, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("strict", [True, False])
def test_hv_count_kernel(strict):
    from evoxmi.ops import geom

    g = torch.Generator().manual_seed(3)
    S, P = torch.rand(20000, 3, generator=g), torch.rand(150, 3, generator=g)
    P[5] = S[7]  # exact equality exercises < vs <=
    ref = geom.hv_count(S, P, strict)
    out = geom.hv_count(S.cuda(), P.cuda(), strict).cpu()
    assert torch.equal(out, ref)


@pytest.mark.gpu
def test_hv_contrib_kernel_and_hype_cal_hv():
    from evoxmi import random as rnd
    from evoxmi.algorithms.mo.hype import cal_hv
    from evoxmi.ops import geom

    g = torch.Generator().manual_seed(4)
    S, P = torch.rand(10000, 3, generator=g), torch.rand(100, 3, generator=g) * 0.8
    cnt = geom.hv_count(S, P, False)
    alpha = torch.rand(100, generator=g)
    ref = geom.hv_contrib(S, P, cnt, alpha)
    out = geom.hv_contrib(S.cuda(), P.cuda(), cnt.cuda(), alpha.cuda()).cpu()
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-5)
    # HypE's estimator on the device equals the CPU oracle for the same samples
    key = rnd.PRNGKey(5)
    ref_pt = torch.full((3,), 1.2)
    f_cpu = cal_hv(P, ref_pt, 50, 10000, key)
    f_gpu = cal_hv(P.cuda(), ref_pt.cuda(), 50, 10000, key.cuda()).cpu()
    assert torch.allclose(f_gpu, f_cpu, rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_igd_and_moead_neighbors_use_knn_kernel():
    from evoxmi.algorithms.mo.moead import nearest_neighbors
    from evoxmi.metrics.igd import igd
    from evoxmi.problems.numerical import DTLZ2

    pf = DTLZ2(m=3).pf()
    objs = pf[::7] + 0.01 * torch.rand(pf[::7].shape, generator=torch.Generator().manual_seed(0))
    assert abs(float(igd(objs.cuda(), pf.cuda())) - float(igd(objs, pf))) < 1e-6
    from evoxmi.operators.sampling import UniformSampling

    w = UniformSampling(1000, 3)()[0].float()
    assert torch.equal(nearest_neighbors(w.cuda(), 20).cpu(), nearest_neighbors(w, 20))


# ---------------------------------------------------------------- K16: OpenES noise regeneration
@pytest.mark.gpu
@pytest.mark.parametrize("rows,d,row0", [(4096, 1000, 0), (1000, 6211, 37), (7, 3, 5)])
def test_es_noise_grad_regenerates_ask_noise(rows, d, row0):
    from evoxmi.algorithms.so.es_variants.open_es import _noise_grad, _normal_rows
    from evoxmi.ops import random as rnd

    key = rnd.PRNGKey(rows + d, device=torch.device("cuda"))
    w = torch.randn(rows, generator=torch.Generator().manual_seed(1)).cuda()
    eps = _normal_rows(key, rows, d, row0, torch.device("cuda"))  # what ask() samples
    ref = (eps.double().T @ w.double()).float()
    g = _noise_grad(key, w, d, row0, torch.device("cuda"))
    assert torch.allclose(g, ref, rtol=1e-4, atol=1e-4 * float(ref.abs().max()))


@pytest.mark.gpu
def test_open_es_gpu_matches_stored_noise_update():
    """One OpenES generation on the GPU with regenerated noise equals the update computed
    from the explicitly stored mirrored noise."""
    from evoxmi import random as rnd
    from evoxmi.algorithms import OpenES

    dev = torch.device("cuda")
    algo = OpenES(torch.zeros(300, device=dev), 64, learning_rate=0.1, noise_stdev=0.5)
    st = algo.init(rnd.PRNGKey(3, device=dev))
    pop, st = algo.ask(st)
    f = (pop * pop).sum(1)
    st2 = algo.tell(st, f)
    eps = (pop - st.center) / 0.5
    grad = (eps.T @ f) / 64 / 0.5
    assert torch.allclose(st2.center, st.center - 0.1 * grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("n", [100, 10000, 20000])
def test_sort_ops_under_vmap_and_on_scalars(n):
    """ops.sort under torch.vmap (BatchedRuns: the custom ops have no batching rule, so the
    batched call must take the torch.sort path) and on 0-d keys."""
    from evoxmi.ops import sort

    x = torch.randn(3, n, device="cuda")
    vi = torch.vmap(lambda r: sort.topk(r, 12, largest=False)[1])(x)
    assert torch.equal(vi, torch.sort(x, dim=1, stable=True)[1][:, :12])
    va = torch.vmap(lambda r: sort.argsort(r)[1])(x)
    assert torch.equal(va, torch.sort(x, dim=1, stable=True)[1])
    v, i = sort.argsort(torch.tensor(2.5, device="cuda"))
    assert float(v) == 2.5 and int(i) == 0


@pytest.mark.parametrize("n", [1, 3, 100, 2048, 5000, 10000, 12000, 16383, 16384, 30001, 65536])
@pytest.mark.parametrize("descending", [0, 1])
@pytest.mark.parametrize("kernel", ["radix_argsort_f32", "rank_argsort_f32", "merge_argsort_f32"])
def test_device_argsort_matches_stable_torch_sort(n, descending, kernel):
    from evoxmi.ops import _ext

    if n > 16384 and kernel != "merge_argsort_f32":
        pytest.skip("single-pass kernels stop at 16384 keys")

    g = torch.Generator().manual_seed(n + descending)
    k = torch.randint(0, n // 4 + 1, (2, n), generator=g).float() / 7  # many ties
    if n < 12:
        k = torch.randn(2, n, generator=g)
        ok, oi = getattr(_ext.ops(), kernel)(k.cuda(), descending)
        rv, ri = torch.sort(k, dim=1, descending=bool(descending), stable=True)
        assert torch.equal(oi.cpu().long(), ri) and torch.equal(ok.cpu(), rv)
        return
    k[0, 3] = float("inf")
    k[0, 9] = float("nan")
    k[1, 5] = float("-inf")
    # a NaN with the sign bit set (x86 0/0) must still sort as the largest value, and
    # -0.0 ties with +0.0 (index order), as in torch.sort
    k[0, 11] = torch.tensor([0xFFC00000], dtype=torch.int64).to(torch.int32).view(torch.float32)[0]
    k[1, 6] = -0.0
    k[1, 7] = 0.0
    k[1, 8] = -0.0
    kd = k.cuda()
    ok, oi = getattr(_ext.ops(), kernel)(kd, descending)
    rv, ri = torch.sort(k, dim=1, descending=bool(descending), stable=True)
    assert torch.equal(oi.cpu().long(), ri) and torch.allclose(ok.cpu(), rv, equal_nan=True)


def test_linear_gp_fit_kernel_matches_torch():
    from evoxmi.algorithms.mo.im_moea import linear_gp_fit

    g = torch.Generator().manual_seed(1)
    n = torch.randint(2, 60, (500,), generator=g).double()
    a = torch.rand(500, generator=g, dtype=torch.float64) * n * 4
    b = (torch.rand(500, generator=g, dtype=torch.float64) - 0.5) * a
    c = torch.rand(500, generator=g, dtype=torch.float64) * n * 3 + b * b / a
    v_r, s2_r = linear_gp_fit(a, b, c, n)
    v, s2 = linear_gp_fit(a.cuda(), b.cuda(), c.cuda(), n.cuda())
    assert torch.allclose(v.cpu(), v_r, rtol=1e-5) and torch.allclose(s2.cpu(), s2_r, rtol=1e-5)


def test_eval_monitor_async_host_history_matches_device_history():
    """history_to_host copies on a side stream (async_d2h) while the hipGraph-replayed
    generations continue; the host history equals the device-kept one."""
    from evoxmi.algorithms import CMAES
    from evoxmi.monitors import EvalMonitor
    from evoxmi.problems.numerical import Sphere
    from evoxmi.workflows import StdWorkflow

    m_host, m_dev = EvalMonitor(history_to_host=True), EvalMonitor()
    wf = StdWorkflow(CMAES(torch.zeros(32, device="cuda") + 3, 1.0, pop_size=64), Sphere(), monitors=[m_host, m_dev], graph=True)
    st = wf.init(rnd.PRNGKey(0, device="cuda"))
    for _ in range(6):
        st = wf.step(st)
    hh, hd = m_host.get_history(), m_dev.get_history()
    assert len(hh) == len(hd) >= 6
    for a, b in zip(hh, hd):
        assert not a.is_cuda and torch.equal(a, b.cpu())


def test_d2h_copier_releases_device_staging_at_flush():
    """A flushed snapshot group keeps no device staging chunk alive until the host entry is
    read (a history read only at the end of a run must not also sit on the device)."""
    from evoxmi.monitors.async_d2h import D2HCopier

    cp = D2HCopier(flush_every=4)
    xs = [torch.full((1000,), float(i), device="cuda") for i in range(8)]
    pend = [cp.submit(x) for x in xs]
    assert all(p.group is None or p.group.dev_buf is None for p in pend)  # both groups flushed
    assert [float(p.get()[0]) for p in pend] == [float(i) for i in range(8)]


@pytest.mark.parametrize("K,D", [(5000, 1000), (7, 33), (130, 257)])
def test_weighted_rowsum_kernel(K, D):
    from evoxmi.ops.reduce import weighted_rowsum

    g = torch.Generator().manual_seed(K)
    X = torch.randn(K + 50, D, generator=g)
    idx = torch.randperm(K + 50, generator=g)[:K].to(torch.int32)
    w = torch.rand(K, generator=g)
    sub = torch.randn(D, generator=g)
    ref = (w.double()[:, None] * (X[idx.long()].double() - sub.double())).sum(0)
    out = weighted_rowsum(X.cuda(), idx.cuda(), w.cuda(), sub.cuda(), K).cpu()
    assert torch.allclose(out.double(), ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("fn", [1, 4])
@pytest.mark.parametrize("N,D", [(10000, 1000), (700, 128), (300, 20), (257, 64)])
def test_cec_rotation_rowterms_epilogue_matches_cpu(fn, N, D):
    """K6: F1 (Zakharov) / F4 (Rastrigin) evaluated from the rotation GEMM's row-terms epilogue
    (the rotated population is never written) vs the fp64 CPU evaluation of the same function."""
    from evoxmi.ops import _ext
    from evoxmi.problems.numerical import CEC2022TestSuit

    from evoxmi import config

    p = CEC2022TestSuit.create(fn)
    g = torch.Generator().manual_seed(N + D)
    X = (torch.rand(N, D, generator=g) * 40 - 20).float()
    ref, _ = p.evaluate(None, X.double())
    with config.override(cec_fused=1):
        out, _ = p.evaluate(None, X.cuda())
    fused = int(_ext.ops().gemm_ks_tile(N, D, 0)) in (4, 8) and D % 4 == 0
    assert out.shape == (N,) and torch.isfinite(out).all()
    torch.testing.assert_close(out.cpu().double(), ref.double(), rtol=2e-4, atol=1e-3)
    if fused:  # the bench shape must take the fused path
        assert N != 10000 or int(_ext.ops().gemm_ks_tile(N, D, 0)) == 8


@pytest.mark.parametrize("col0,own,d", [(0, 30, 30), (7, 11, 30), (13, 17, 30), (1, 1000, 1003)])
def test_pso_column_block_update_matches_unsharded(col0, own, d):
    """P2 state sharding: the column-block PSO kernel (Philox counter = row·d_total + column)
    reproduces the corresponding columns of the unsharded update bit for bit."""
    from evoxmi.ops.pso import pso_update

    n = 37
    g = torch.Generator().manual_seed(col0 + own)
    pop, vel, lbl = (torch.rand(n, d, generator=g) * 10 - 5 for _ in range(3))
    lbf, fit = torch.rand(n, generator=g), torch.rand(n, generator=g)
    gbl, lb, ub = torch.rand(d, generator=g), torch.full((d,), -4.0), torch.full((d,), 4.0)
    kp, kg = rnd.PRNGKey(11), rnd.PRNGKey(12)
    cu = lambda t: t.cuda()
    full = pso_update(cu(pop), cu(vel), cu(lbl), cu(lbf), cu(fit), cu(gbl), cu(kp), cu(kg), 0.6, 2.5, 0.8, cu(lb), cu(ub))
    c = slice(col0, col0 + own)
    part = pso_update(cu(pop[:, c].contiguous()), cu(vel[:, c].contiguous()), cu(lbl[:, c].contiguous()), cu(lbf), cu(fit),
                      cu(gbl[c].contiguous()), cu(kp), cu(kg), 0.6, 2.5, 0.8, cu(lb[c].contiguous()), cu(ub[c].contiguous()),
                      col0=col0, d_total=d)
    for a, b in zip(full[:3], part[:3]):
        assert torch.equal(a[:, c], b)
    assert torch.equal(full[3], part[3])
    cpu = pso_update(pop[:, c].contiguous(), vel[:, c].contiguous(), lbl[:, c].contiguous(), lbf, fit, gbl[c].contiguous(), kp, kg,
                     0.6, 2.5, 0.8, lb[c].contiguous(), ub[c].contiguous(), col0=col0, d_total=d)
    assert torch.allclose(cpu[0], part[0].cpu(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("col0,own,d", [(0, 30, 30), (7, 11, 30), (29, 1, 30), (3, 500, 1001)])
@pytest.mark.parametrize("mode", [0, 1])
def test_de_trial_column_block_matches_unsharded(col0, own, d, mode):
    """P2 state sharding for DE: a column block of the trial vectors (global Philox word, j_rand
    and exponential window) equals those columns of the unsharded fused trials, and the CPU
    oracle of the block."""
    from evoxmi.ops.evo import de_trial

    R, rows, K = 23, 40, 3
    g = torch.Generator().manual_seed(col0 + own + mode)
    P = torch.rand(rows, d, generator=g) * 10 - 5
    idx = torch.randint(0, rows, (R, K), generator=g, dtype=torch.int32)
    coef = torch.rand(R, K, generator=g)
    cur = torch.arange(R, dtype=torch.int32)
    md = torch.full((R,), mode, dtype=torch.int32)
    CR = torch.rand(R, generator=g)
    jr = torch.randint(0, d, (R,), generator=g, dtype=torch.int32)
    L = torch.randint(0, d, (R,), generator=g, dtype=torch.int32)
    lb, ub = torch.full((d,), -4.0), torch.full((d,), 4.0)
    key = rnd.PRNGKey(7)
    cu = lambda t: t.cuda()
    full = de_trial(cu(key), cu(P), cu(idx), cu(coef), cu(cur), cu(md), cu(CR), cu(jr), cu(L), cu(lb), cu(ub))
    c = slice(col0, col0 + own)
    part = de_trial(cu(key), cu(P[:, c].contiguous()), cu(idx), cu(coef), cu(cur), cu(md), cu(CR), cu(jr), cu(L), cu(lb[c].contiguous()),
                    cu(ub[c].contiguous()), col0=col0, d_total=d)
    assert torch.equal(full[:, c], part)
    cpu = de_trial(key, P[:, c].contiguous(), idx, coef, cur, md, CR, jr, L, lb[c].contiguous(), ub[c].contiguous(), col0=col0, d_total=d)
    assert torch.allclose(cpu, part.cpu(), rtol=1e-5, atol=1e-5)


def test_cec_basic_fused_clamp_matches_where():
    """The f < 1e-8 → 0 rule of the CEC'22 evaluation fused into cec_basic_kernel (clamp > 0); clamp = 0
    leaves negative values alone; NaN rows stay NaN."""
    from evoxmi.ops import numerical as nops
    from evoxmi.problems.numerical.cec2022 import SCHWEFEL, ZAKHAROV

    g = torch.Generator().manual_seed(3)
    Z = torch.randn(8, 64, generator=g)
    Z[0] = 0.0
    Z[1] = 1e-9  # f ≈ (0.5·Σ(j+1)·1e-9)² ≈ 1e-12 < 1e-8
    Z[2, 5] = float("nan")
    Zd = Z.cuda()
    plain = nops.cec_basic(Zd, ZAKHAROV, None, 0, 64).cpu()
    fused = nops.cec_basic(Zd, ZAKHAROV, None, 0, 64, clamp=1e-8).cpu()
    ref = torch.where(plain < 1e-8, torch.zeros_like(plain), plain)
    assert torch.equal(fused[~torch.isnan(ref)], ref[~torch.isnan(ref)]) and torch.isnan(fused[2])
    assert fused[0] == 0 and fused[1] == 0
    s = nops.cec_basic(Zd * 50, SCHWEFEL, None, 0, 64).cpu()
    assert torch.equal(nops.cec_basic(Zd * 50, SCHWEFEL, None, 0, 64, clamp=0.0).cpu()[~torch.isnan(s)], s[~torch.isnan(s)])


@pytest.mark.gpu
@pytest.mark.parametrize("d,world", [(32, 2), (30, 3), (1000, 8)])
def test_sbx_pm_kernels_column_blocks(d, world):
    """evo_ops.hip sbx / pm with (col0, dtot): every column block equals those columns of the
    full-width kernels (both the 4-gene Philox path and the scalar path) and the CPU oracle."""
    from evoxmi.operators import crossover, mutation
    from evoxmi.parallel.context import balanced_slices

    x = torch.rand(64, d, generator=torch.Generator().manual_seed(2)).cuda()
    lb, ub = torch.zeros(d, device="cuda"), torch.ones(d, device="cuda")
    key = rnd.PRNGKey(9, device="cuda")
    full_x = crossover.simulated_binary(key, x)
    full_m = mutation.polynomial(key, full_x, (lb, ub))
    assert torch.allclose(full_x.cpu(), crossover.simulated_binary(key.cpu(), x.cpu()), atol=1e-5)
    for c0, own in balanced_slices(d, world):
        blk = crossover.simulated_binary(key, x[:, c0 : c0 + own].contiguous(), cols=(c0, d))
        assert torch.equal(blk, full_x[:, c0 : c0 + own])
        mb = mutation.polynomial(key, blk, (lb[c0 : c0 + own], ub[c0 : c0 + own]), cols=(c0, d))
        assert torch.equal(mb, full_m[:, c0 : c0 + own])


@pytest.mark.gpu
@pytest.mark.parametrize("d", [6472, 37])
@pytest.mark.parametrize("mirrored", [True, False])
def test_openes_population_kernel_matches_noise_rows(d, mirrored):
    """rng.hip es_population_kernel: center + σ·ε (mirrored halves negated) in one pass equals
    the materialised form center + σ·noise_rows bit for bit, for whole and partial row ranges."""
    from evoxmi.algorithms import OpenES

    pop = 64
    center = torch.randn(d, generator=torch.Generator().manual_seed(3)).cuda()
    es = OpenES(center, pop, 0.05, 0.1, mirrored_sampling=mirrored)
    key = rnd.PRNGKey(11, device="cuda")
    for start, size in [(0, pop), (5, 40), (pop // 2, pop // 2)]:
        ref = center[None, :] + es.noise_stdev * es._noise_rows(key, start, size, center.device)
        got = es._population_rows(key, center, start, size)
        assert torch.equal(got, ref), (start, size)


@pytest.mark.parametrize("keep", [0, 1])
def test_cma_eig_out_selects_the_warm_start_on_the_keep_word(keep):
    """Round 6: the device eigensolver's restore copy is folded into cma_eig_out — while the keep
    word is 0 (diverged / no iteration ran) the basis is the warm start B_alt (here the output
    buffer itself, as under capture), else the solver's basis; D = sqrt(w), B/D by columns."""
    d = 96
    g = torch.Generator().manual_seed(3)
    Bp = torch.randn(d, d, generator=g).cuda()
    Bw = torch.randn(d, d, generator=g).cuda()
    w = (torch.rand(d, generator=g) + 0.1).cuda()
    out = Bw.clone()  # B_out aliases B_alt
    kw = torch.full((1,), keep, dtype=torch.int32, device="cuda")
    B, D, BD = _ext.ops().cma_eig_out(Bp, w, d, out, out, kw)
    ref = Bp if keep else Bw
    assert B.data_ptr() == out.data_ptr()
    assert torch.equal(B, ref)
    assert torch.allclose(D, w.sqrt())
    assert torch.allclose(BD, ref / w.sqrt()[None, :], rtol=1e-6, atol=1e-7)


def test_cma_center_rows_augmented_product_carries_the_mean_shift():
    """Round 6: the rank-μ rows augmented by σ·sqrt(wᵢ) — the (d+1)-square product's last row is
    Σ wᵢ (xᵢ − m) and its leading block Σ wᵢ yᵢ yᵢᵀ (fp64 reference)."""
    from evoxmi.ops.linalg import mm

    d, n, K = 1000, 300, 120
    g = torch.Generator().manual_seed(4)
    pop = (torch.randn(n, d, generator=g) * 3).cuda()
    mean = torch.randn(d, generator=g).cuda()
    sigma = torch.tensor([1.7]).cuda()
    rows = torch.randperm(n, generator=g)[:K].to(torch.int32).cuda()
    w = torch.rand(K, generator=g).cuda()
    w = w / w.sum()
    Yw = _ext.ops().cma_center_rows(pop, rows, mean, sigma, w, True)
    assert Yw.shape == (K, d + 1) and Yw.stride(0) % 4 == 0
    S = mm(Yw, Yw, ta=True, mode=1, out=torch.empty(d + 1, Yw.stride(0), device="cuda")[:, : d + 1])
    x = pop[rows.long()].double() - mean.double()
    dm = (w.double()[:, None] * x).sum(0)
    y = x / 1.7
    Sref = (y * w.double()[:, None]).T @ y
    assert torch.allclose(S[d, :d].double(), dm, rtol=1e-5, atol=1e-5)
    assert torch.allclose(S[:d, :d].double(), Sref, rtol=1e-5, atol=3e-5)
