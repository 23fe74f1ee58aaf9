"""Sorted-block refinement eigensolver (evoxmi/ops/sbr.py, csrc/kernels/eigh_sbr.hip).

CPU tests pin the algorithm (torch reference) on CMA-ES-like matrices; GPU tests compare
each HIP kernel with that fp32 reference and check that the hybrid solver converges to
the configured tolerance on every generation of a CMA-ES run at the north-star shape,
with best-fitness trajectories matching the library eigensolver (reference:
``cma_es.py:155-160,193-198`` decomposes with jnp.linalg.eigh every generation)."""
import math

import pytest
import torch

from evoxmi.ops import sbr


def _cma_like(n, gens, seed=0, dev="cpu"):
    """C after `gens` rank-μ updates (random selection, μ_eff ≈ 2.5·n, cμ as in CMA-ES at
    λ = 10n) and the previous generation's exact eigenbasis."""
    g = torch.Generator(device=dev).manual_seed(seed)
    mu = 5 * n
    w = math.log(mu + 0.5) - torch.log(torch.arange(1, mu + 1, dtype=torch.float64))
    w = (w / w.sum()).to(dev)
    mueff = float(w.sum() ** 2 / (w**2).sum())
    cmu = 2 * (mueff - 2 + 1 / mueff) / ((n + 2) ** 2 + mueff)
    C = torch.eye(n, dtype=torch.float64, device=dev)
    Bprev = C.clone()
    for _ in range(gens):
        L = torch.linalg.cholesky(C)
        z = torch.randn(mu, n, generator=g, dtype=torch.float64, device=dev)
        y = z @ L.T
        Bprev = torch.linalg.eigh(C)[1]
        C = (1 - cmu) * C + cmu * (y.T * w) @ y
    return C.float(), Bprev.float()


def _offrel(A):
    d = torch.diagonal(A)
    return float(torch.linalg.matrix_norm(A - torch.diag(d)) / torch.linalg.vector_norm(d))


def test_round_robin_pairs_cover_all_pairs_once():
    seen = set()
    for p, q in sbr._rr_rounds(64):
        ps = p.tolist() + q.tolist()
        assert len(set(ps)) == 64  # disjoint within a round
        for a, b in zip(p.tolist(), q.tolist()):
            assert a < b and (a, b) not in seen
            seen.add((a, b))
    assert len(seen) == 64 * 63 // 2


@pytest.mark.parametrize("n,off", [(200, 0), (200, 32), (64, 0), (30, 32)])
def test_block_layout(n, off):
    st = sbr.block_starts(n, off)
    assert st[0] == 0 and st[-1] == n and all(b - a <= 64 for a, b in zip(st, st[1:]))
    assert sbr.nblocks(n, off) == len(st) - 1


def test_block_solve_reference_diagonalises_small_matrix():
    torch.manual_seed(0)
    M = torch.randn(40, 40)
    A = M @ M.T / 40
    perm, Q, dq = sbr.block_solve_ref(A, 0, 10)
    p = perm.long()
    A1 = Q[0, :40, :40].T @ A[p][:, p] @ Q[0, :40, :40]
    assert _offrel(A1) < 1e-5
    assert torch.allclose(torch.diagonal(A1), dq, atol=1e-4)
    assert torch.allclose(Q[0].T @ Q[0], torch.eye(64), atol=1e-5)


def test_refinement_converges_on_cma_like_matrix_cpu():
    C, B = _cma_like(256, 30)
    w, Bn, info = sbr.eigh_warm(C, B)
    assert info.off_rel <= 1e-5, info
    A = Bn.T @ C @ Bn
    assert _offrel(A) <= 2e-5
    assert torch.linalg.matrix_norm(Bn.T @ Bn - torch.eye(256)) < 1e-4
    assert torch.allclose(torch.sort(w).values, torch.linalg.eigvalsh(C.double()).float(), atol=1e-5)



@pytest.mark.parametrize("n,shift", [(200, 0), (200, 8), (37, 8), (1000, 8)])
def test_shifted_layout_reference(n, shift):
    """16-block layout: perm is the stable argsort rolled by the shift, every block is
    diagonalised by the reference sweeps and Bq = B[:, perm]·blockdiag(Q)."""
    C, B = _cma_like(n, 3, seed=n) if n <= 200 else (None, None)
    if C is None:
        torch.manual_seed(0)
        M = torch.randn(n, n)
        C = M @ M.T / n
        B = torch.linalg.qr(torch.randn(n, n))[0]
    A = sbr.sym_product(C, B)
    perm, Q, dq = sbr.block_solve16_ref(A, shift, 6)
    ref = torch.roll(torch.argsort(torch.diagonal(A), stable=True), -shift)
    assert torch.equal(perm.long(), ref)
    Qf = sbr._blockdiag16(Q, n)
    A1 = Qf.T @ A[perm.long()][:, perm.long()] @ Qf
    blk = torch.arange(n) // 16
    inblock = (blk[:, None] == blk[None, :]) & ~torch.eye(n, dtype=torch.bool)
    assert float(A1[inblock].abs().max()) < 1e-5 * float(A.abs().max())
    assert torch.allclose(torch.diagonal(A1), dq, atol=1e-5)
    assert torch.allclose(sbr.bq16_ref(B, perm, Q), B[:, perm.long()] @ Qf)


def test_refinement_block16_converges_cpu():
    C, B = _cma_like(256, 30)
    w, Bn, info = sbr.eigh_warm(C, B, sbr.SBRConfig(block=16))
    assert info.off_rel <= 1e-5, info
    assert _offrel(Bn.T @ C @ Bn) <= 2e-5


def test_near_only_iteration_is_not_repeated():
    """A near-only iteration (no far step) that misses the tolerance is followed by a
    full one: the driver must not stall on far-pair residue."""
    C, B = _cma_like(256, 8, seed=3)
    w, Bn, info = sbr.eigh_warm(C, B, sbr.SBRConfig(block=16, near_only=1e6))
    assert info.off_rel <= 1e-5 and info.refine_iters < 16, info


# ------------------------------------------------------------------ GPU
gpu = pytest.mark.gpu


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30)).item()


@gpu
@pytest.mark.parametrize("n", [200, 1000])
def test_sbr_stats_kernel(n):
    torch.manual_seed(n)
    A = torch.randn(n, n)
    A = A + A.T
    out = sbr.stats(A.cuda()).cpu()
    ref = sbr.stats_ref(A)
    assert torch.allclose(out, ref, rtol=1e-9)


@gpu
@pytest.mark.parametrize("n,off", [(1000, 0), (1000, 32), (200, 32), (37, 0)])
def test_sbr_kernels_match_reference(n, off):
    C, B = _cma_like(n, 8, seed=n)
    A = sbr.sym_product(C, B)
    st = sbr.stats_ref(A)
    perm_r, Q_r, dq_r = sbr.block_solve_ref(A, off, 2)
    Ad = A.cuda()
    perm, Q, dq = sbr.block_solve(Ad, off, 2)
    assert torch.equal(perm.cpu(), perm_r)
    # two sweeps leave near-degenerate pairs partially rotated, so individual Q columns are
    # rounding-sensitive; compare what the algorithm relies on: orthogonality, the block
    # off-norm reached, and dq = diag(Qᵀ A_blk Q)
    Q, dq = Q.cpu(), dq.cpu()
    nb = Q.shape[0]
    assert float((Q.transpose(1, 2) @ Q - torch.eye(64)).abs().max()) < 2e-5
    st_ = sbr.block_starts(n, off)
    for k in range(nb):
        m = st_[k + 1] - st_[k]
        idx = perm_r[st_[k] : st_[k + 1]].long()
        S = A[idx][:, idx]
        T = Q[k, :m, :m].T @ S @ Q[k, :m, :m]
        T_r = Q_r[k, :m, :m].T @ S @ Q_r[k, :m, :m]
        off_k = torch.linalg.matrix_norm(T - torch.diag(torch.diagonal(T)))
        off_r = torch.linalg.matrix_norm(T_r - torch.diag(torch.diagonal(T_r)))
        assert off_k <= 1.5 * off_r + 1e-6 * torch.linalg.matrix_norm(S)
        assert torch.allclose(torch.diagonal(T), dq[st_[k] : st_[k + 1]], atol=2e-5)
    # downstream kernels on identical inputs
    X = sbr.far(Ad, off, perm_r.cuda(), Q_r.cuda(), dq_r.cuda(), st.cuda(), 0.3).cpu()
    X_r = sbr.far_ref(A, off, perm_r, Q_r, dq_r, st, 0.3)
    assert (X.abs() > 0).sum() == (X_r.abs() > 0).sum()
    assert _rel(X, X_r) < 1e-4
    Bq = sbr.bq(B.cuda(), off, perm_r.cuda(), Q_r.cuda()).cpu()
    assert _rel(Bq, sbr.bq_ref(B, off, perm_r, Q_r)) < 1e-5



@gpu
@pytest.mark.parametrize("sb", [16, 32])
@pytest.mark.parametrize("n,shift", [(1000, 0), (1000, 8), (200, 8), (37, 8), (17, 0), (2100, 8)])  # n ≤ 2048: rank fused into the block kernel
def test_sbr16_kernels_match_reference(n, shift, sb):
    C, B = _cma_like(n, 8, seed=n)
    A = sbr.sym_product(C, B)
    st = sbr.stats_ref(A)
    perm_r, Q_r, dq_r = sbr.block_solve16_ref(A, shift, 2, sb)
    Ad = A.cuda()
    perm, Q, dq = sbr.block_solve(Ad, shift, 2, bk=sb)
    assert torch.equal(perm.cpu(), perm_r)
    Q, dq = Q.cpu(), dq.cpu()
    assert float((Q.transpose(1, 2) @ Q - torch.eye(sb)).abs().max()) < 4e-6
    p = perm_r.long()
    for k in range(Q.shape[0]):
        idx = p[sb * k : sb * (k + 1)]
        m = idx.numel()
        S = A[idx][:, idx]
        T = Q[k, :m, :m].T @ S @ Q[k, :m, :m]
        T_r = Q_r[k, :m, :m].T @ S @ Q_r[k, :m, :m]
        off_k = torch.linalg.matrix_norm(T - torch.diag(torch.diagonal(T)))
        off_r = torch.linalg.matrix_norm(T_r - torch.diag(torch.diagonal(T_r)))
        assert off_k <= 1.5 * off_r + 1e-6 * torch.linalg.matrix_norm(S)
        assert torch.allclose(torch.diagonal(T), dq[sb * k : sb * k + m], atol=2e-5)
    X = sbr.far(Ad, shift, perm_r.cuda(), Q_r.cuda(), dq_r.cuda(), st.cuda(), 0.5, bk=sb).cpu()
    X_r = sbr.far16_ref(A, perm_r, Q_r, dq_r, st, 0.5)
    assert (X.abs() > 0).sum() == (X_r.abs() > 0).sum()
    assert _rel(X, X_r) < 1e-4
    Bq = sbr.bq(B.cuda(), shift, perm_r.cuda(), Q_r.cuda(), bk=sb).cpu()
    assert _rel(Bq, sbr.bq16_ref(B, perm_r, Q_r)) < 1e-5


@gpu
@pytest.mark.parametrize("gens", [1, 4, 15, 40])
def test_sbr_eigh_converges_at_north_star_size(gens):
    """Every generation's decomposition reaches the tolerance (early generations need the
    Jacobi hand-off, later ones refine directly)."""
    C, B = _cma_like(1000, gens, seed=gens, dev="cuda")
    w, Bn, info = sbr.eigh_warm(C, B)
    assert info.off_rel <= 1e-5, info
    A = (Bn.T.double() @ C.double() @ Bn.double())
    assert _offrel(A) <= 2e-5
    assert float(torch.linalg.matrix_norm(Bn.T.double() @ Bn.double() - torch.eye(1000, device="cuda", dtype=torch.float64))) < 1e-3
    ev = torch.linalg.eigvalsh(C.double())
    # eigenvalue error ≤ ‖offdiag‖₂ (first order, clustered spectrum)
    assert float((torch.sort(w.double()).values - ev).abs().max()) < 5e-5


@gpu
def test_cmaes_trajectories_sbr_vs_library_eigh():
    """CMA-ES λ = 10⁴, d = 1000 for 100 generations with the converged SBR solver and with
    rocSOLVER eigh: every SBR decomposition meets the tolerance and the runs make the same
    progress.  Progress is the objective at the distribution mean on the (axis-scaled)
    Ellipsoid, which CMA-ES must learn through its eigenbasis; best-so-far on CEC'22 F1 is
    no measure here — it freezes at the luckiest early sample while σ adapts, and on F1
    even the mean's value swings by orders of magnitude (tools/traj_probe.py).  Two
    decompositions that agree to 1e-5 still make the runs drift apart chaotically (≈10 %
    per seed after 60 generations), so the comparison uses the median over ten seeds (round 6:
    five-seed medians of the same solver spread over ±3 % between disjoint seed sets, the size of
    the 5 % bound — profiles/r6_parity_15_seeds.txt)."""
    import statistics

    from evoxmi import config as cfg
    from evoxmi import random as rnd
    from evoxmi.algorithms import CMAES
    from evoxmi.problems.numerical import Ellipsoid
    from evoxmi.workflows import StdWorkflow

    def traj(impl, seed):
        # a schedule long enough for the cold-start generations (≤ 12 iterations): this test
        # pins every decomposition to the tolerance; the default schedule (8) caps the first
        # two generations (tests/test_sbr_device_gpu.py covers the cap)
        with cfg.override(eigh=impl, sbr_device_iters=16):
            center = (torch.rand(1000, generator=torch.Generator().manual_seed(1)) * 10 - 5).cuda()
            algo = CMAES(center_init=center, init_stdev=1.0, pop_size=10000)
            prob = Ellipsoid()
            # rocSOLVER syevd is not hipGraph-capturable: the library run steps eagerly
            wf = StdWorkflow(algo, prob, graph=(impl == "sbr"))
            st = wf.init(rnd.PRNGKey(seed, device=torch.device("cuda")))
            pst = st.get_child_state("problem")
            f, offs = [], []
            for _ in range(100):
                st = wf.step(st)
                a = st.get_child_state("algorithm")
                f.append(float(prob.evaluate(pst, a.mean.reshape(1, -1))[0][0]))
                if impl == "sbr":
                    offs.append(float(a.eig_stats[0]))
            return f, offs

    runs = {impl: [traj(impl, s) for s in range(7, 17)] for impl in ("sbr", "torch")}
    offs = [o for f, oo in runs["sbr"] for o in oo]
    assert max(offs) <= 1e-5, max(offs)
    med = {impl: [statistics.median(r[0][g] for r in runs[impl]) for g in range(100)] for impl in runs}
    logr = [abs(math.log(med["sbr"][g] / med["torch"][g])) for g in range(10, 100)]
    assert statistics.median(logr) < math.log(1.05), (statistics.median(logr), med["sbr"][::10], med["torch"][::10])
    prog = {impl: math.log(med[impl][10] / med[impl][99]) for impl in med}
    assert prog["torch"] > 1.0 and abs(prog["sbr"] / prog["torch"] - 1) < 0.05, prog


@gpu
def test_damping_kernel_matches_torch_power_iteration():
    torch.manual_seed(5)
    n = 1000
    M = torch.randn(n, n) * 1e-3
    X = M - M.T
    X2 = (X @ X).cuda()
    V = sbr._probe_vectors(n, "cuda")
    a = float(sbr.damping(X2, 0.05))
    X2c, Vc = X2.cpu().double(), V.cpu().double()
    V1 = -(X2c @ Vc)
    V2 = -(X2c @ V1)
    V3 = -(X2c @ V2)
    lam = float((V3.norm(dim=0) / V2.norm(dim=0)).max())
    ref = min(1.0, 0.05 / math.sqrt(lam))
    assert abs(a - ref) <= 1e-4 * ref


@gpu
def test_sbr_eigh_is_deterministic():
    """Same inputs, fresh plans ⇒ bitwise identical decompositions (graph captures on first
    use of an iteration variant must not apply the iteration twice)."""
    C, B = _cma_like(1000, 6, seed=3, dev="cuda")
    outs = [sbr.eigh_warm(C, B, sbr.SBRConfig(), plans={}) for _ in range(3)]
    for w, Bn, info in outs[1:]:
        assert torch.equal(Bn, outs[0][1]) and info.refine_iters == outs[0][2].refine_iters


@gpu
@pytest.mark.parametrize("order", [4, 6])
def test_taylor_exponential_kernels(order):
    torch.manual_seed(order)
    n = 300
    M = torch.randn(n, n) * 0.003  # ‖X‖₂ ≈ 0.15: Taylor-4 is orthogonal to ~1e-6 there
    X = M - M.T
    X2 = X @ X
    alpha = torch.tensor([0.7])
    f = sbr.expm_taylor4 if order == 4 else sbr.expm_taylor6
    ref = f(X, X2, alpha)
    out = f(X.cuda(), X2.cuda(), alpha.cuda()).cpu()
    assert _rel(out, ref) < 1e-5
    assert float((ref.T @ ref - torch.eye(n)).abs().max()) < 1e-5  # orthogonal to the order's truncation
