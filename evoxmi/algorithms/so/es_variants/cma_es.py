"""CMA-ES family: CMAES, SepCMAES, IPOPCMAES, BIPOPCMAES.

Parity: reference ``algorithms/so/es_variants/cma_es.py`` (Hansen tutorial
CMA-ES, ``:33-198``; SepCMAES ``:202-255``; IPOP/BIPOP ``:259-390``).  Default
λ = 4 + ⌊3 ln d⌋, μ = λ/2, log weights, and the same learning-rate formulas, so
at the north-star shape (d = 1000, λ = 10 000) μ_eff ≈ 2508.6, c1 ≈ 2.0e-6,
cμ ≈ 4.98e-3 and the eigendecomposition runs every generation.

MI355X execution of one generation on a GPU (everything stays in HBM, no host
synchronisation, hipGraph-capturable):

* ``ask``: Philox normals (``rng.hip``) → ONE f32 GEMM ``X = mean + σ·Z (B∘D)ᵀ``
  on the framework kernel (``gemm_ks.hip``: σ as a device scale, ``mean`` as the
  bias epilogue).
* ``tell``: argsort of the fitness; the weighted mean is a gathered weighted row
  sum (``reduce.hip``); the rank-μ update ``Σ wᵢ yᵢ yᵢᵀ`` is a symmetric-output
  framework GEMM (upper tiles only) on the materialised ``Yw = (x_sel − m)/σ·√w``
  (``cma_center_rows``), or the older framework GEMM whose prologue *gathers* the
  selected rows (``EVOXMI_PLAIN_GEMM`` ≠ evoxmi/blas);
  converged sorted-block-refinement ``eigh`` (:mod:`evoxmi.ops.sbr`); ``invsqrtC``
  = (B/D)Bᵀ as a symmetric-output GEMM.  ``EVOXMI_PLAIN_GEMM=blas`` swaps the plain
  products for hipBLASLt (an A/B baseline only).
* Sharded (``ask_sharded``/``tell_sharded``): each rank generates only its rows
  (Philox counters are global row indices, so 1/2/4/8 GPUs sample the same
  population), fitness is all-gathered, and each rank all-reduces its partial
  weighted sums (d + d² floats) over RCCL; the state stays replicated.
"""
from __future__ import annotations

import math

import torch

from ....core import Algorithm, State
from ....ops import random as rnd
from ....ops.eigh import sbr_phase, symmetrize_upper, warm_eigh
from ....runtime import host_phase
from ....utils import profiling
from .... import config
from ....ops import linalg
from ....parallel.dim_sharded import ColumnSeparable
from ....ops.linalg import Operand, gemm, mm, plain_nt
from ....ops.reduce import weighted_rowsum
from ....ops.sort import argsort, argsort_i32


def _default_weights(mu: int):
    w = math.log(mu + 0.5) - torch.log(torch.arange(1, mu + 1, dtype=torch.float64))
    return (w / w.sum()).to(torch.float32)


class CMAES(Algorithm):
    # fields that differ across ranks under the sharded protocol (excluded from replica checks)
    rank_local_fields = ("population",)

    def __init__(self, center_init, init_stdev, pop_size=None, recombination_weights=None, cm=1, eig_sweeps=None):
        super().__init__()
        self.center_init = center_init
        assert init_stdev > 0, "Expect variance to be a non-negative float"
        self.init_stdev = float(init_stdev)
        self.dim = center_init.shape[0]
        self.cm = cm
        self.eig_sweeps = eig_sweeps
        self.pop_size = 4 + math.floor(3 * math.log(self.dim)) if pop_size is None else pop_size
        if recombination_weights is None:
            self.mu = self.pop_size // 2
            self.weights = _default_weights(self.mu)
        else:
            rw = torch.as_tensor(recombination_weights, dtype=torch.float32)
            assert bool((rw[1:] <= rw[:-1]).all()), "recombination_weights must be non-increasing"
            assert abs(float(rw.sum()) - 1) < 1e-6, "sum of recombination_weights must be 1"
            assert bool((rw > 0).all()), "recombination_weights must be positive"
            self.mu = rw.shape[0]
            assert self.mu <= self.pop_size
            self.weights = rw
        self.weights = self.weights.to(center_init.device)
        self._set_rates()
        # iteration plans of the converged eigensolver, private to this optimiser run
        # (evoxmi.ops.sbr.eigh_warm): results depend only on the run's own history
        self._eig_plans = {}

    def _set_rates(self):
        w = self.weights.double()
        d = self.dim
        self.mueff = float(w.sum() ** 2 / (w**2).sum())
        self.cc = (4 + self.mueff / d) / (d + 4 + 2 * self.mueff / d)
        self.cs = (2 + self.mueff) / (d + self.mueff + 5)
        self.c1 = 2 / ((d + 1.3) ** 2 + self.mueff)
        self.cmu = min(1 - self.c1, 2 * (self.mueff - 2 + 1 / self.mueff) / ((float(d) + 2) ** 2 + self.mueff))
        self.damps = 1 + 2 * max(0, math.sqrt((self.mueff - 1) / (d + 1)) - 1) + self.cs
        self.chiN = d**0.5 * (1 - 1 / (4 * d) + 1 / (21 * d**2))
        self.decomp_per_iter = max(int(math.floor(1 / (self.c1 + self.cmu) / d / 10)), 1)

    # ------------------------------------------------------------------ state
    def setup(self, key):
        dev = self.center_init.device
        d = self.dim
        self._sched_reset()
        B = torch.eye(d, device=dev)
        C = torch.eye(d, device=dev)
        return State(
            pc=torch.zeros(d, device=dev),
            ps=torch.zeros(d, device=dev),
            B=B,
            D=torch.ones(d, device=dev),
            C=C,
            count_eigen=torch.zeros((), dtype=torch.int64, device=dev),
            count_iter=torch.zeros((), dtype=torch.int64, device=dev),
            invsqrtC=C.clone(),
            mean=self.center_init.to(torch.float32).clone(),
            sigma=torch.tensor(self.init_stdev, dtype=torch.float32, device=dev),
            key=key.to(dev),
            population=torch.zeros((self.pop_size, d), device=dev),
            # last decomposition: [relative off-norm, Jacobi sweeps, refinement iterations, fallback]
            eig_stats=torch.zeros(4, dtype=torch.float64, device=dev),
        )

    # ------------------------------------------------------------------ step variants
    def _device_eigh(self) -> bool:
        return (self.center_init.is_cuda and self.decomp_per_iter == 1 and config.get("cma_fused") and config.get("eigh") == "sbr"
                and config.get("sbr_mode") == "device" and self.dim % 4 == 0 and self.dim <= 8192)

    # ------------------------------------------------------------------ eigensolver schedule
    # The device eigensolver runs a fixed number of refinement slots per generation (a skipped
    # slot still costs its launch boundaries — ≈10 kernels, ≈45 µs in graph replay), in four captured
    # graph variants: "cold" (sbr_cold_iters slots — the first solves from C = I need 10-12
    # iterations), None (the warm schedule, sbr_device_iters), "warm6" (one slot fewer: most warm
    # solves take 5) and "late" (sbr_late_iters, lean: settled solves take 4).
    # Which one a generation replays is chosen from MEASURED convergence, not from the
    # generation index (round 6; round 5 switched at fixed generations 4 and 24 tuned on one
    # trajectory):
    #
    # * each solve writes [off_rel, status, iterations, fallback, seq] into a host-mapped pinned
    #   ring inside the generation (one single-thread kernel of its graph) and an event is
    #   recorded after the step; choosing the variant of a step reads the solve of the step
    #   ESC_LAG = 2 back (waiting on that step's event never idles the GPU while the step after
    #   it is queued; no .item(), no device synchronize) — a fixed lag, so the choice and the
    #   run are deterministic;
    # * a solve that capped or fell back, or that converged only in its schedule's last slot,
    #   moves the schedule one level up from the level it ran at (late → warm → cold); a solve
    #   that would not fit the current level with one slot to spare moves it back to the
    #   level it ran at (the "first slow solve" rule);
    # * DOWN_STREAK consecutive solves at the current level that would have fitted the next
    #   shorter schedule with one slot to spare move it one level down.
    LEVELS = ("late", "warm6", None, "cold")
    TOP = len(LEVELS) - 1
    ESC_LAG = 2
    ESC_RING = 16
    DOWN_STREAK = 2

    def _sched(self):
        sc = self.__dict__.get("_sched_state")
        if sc is None:
            sc = self._sched_state = self._sched_fresh()
        return sc

    @staticmethod
    def _sched_fresh():
        from collections import deque

        return {"level": CMAES.TOP, "streak": 0, "enqueued": 0, "checked": -1, "pending": deque(), "last": CMAES.TOP, "escalations": 0,
                "history": [], "levels": []}

    def _sched_reset(self):
        """A new run (``setup``): the schedule starts cold again and forgets the previous run's
        solves; the device report counter and ring are re-based so slot k again holds solve k."""
        self._sched_state = self._sched_fresh()
        if self.__dict__.get("_eig_seq") is not None:
            self._eig_seq.zero_()
            self._eig_ring.fill_(-1.0)

    def _level_slots(self, level: int) -> int:
        from ....ops.sbr_device import schedule_iters

        return schedule_iters(self.dim, ("late", "warm6", "warm", "cold")[level])

    def graph_variant(self, generation: int):
        """The eigensolver schedule of the next step (see the class comment above): one of
        ``LEVELS``, chosen from the measured convergence of the solve ``ESC_LAG`` steps back."""
        if not self._device_eigh():
            return None
        sc = self._sched()
        self._poll_eig_health(sc)
        sc["last"] = sc["level"]
        return self.LEVELS[sc["level"]]

    def graph_variant_set(self):
        if not self._device_eigh():
            return ()
        return self.LEVELS

    def after_step(self, generation: int) -> None:
        if self.__dict__.get("_eig_ring") is None or not torch.cuda.is_available():
            return
        sc = self._sched()
        ev = torch.cuda.Event()
        ev.record()
        k = sc["enqueued"]
        sc["pending"].append((k, ev, sc["last"]))
        sc["levels"].append(sc["last"])
        del sc["levels"][:-4096]
        sc["enqueued"] = k + 1
        while len(sc["pending"]) > self.ESC_RING // 2:
            sc["pending"].popleft()

    def _report_buffers(self, device):
        """(device counter, host-mapped pinned ring) the solve's last control kernel writes its
        [off_rel, status, iterations, fallback, seq] into (captured into the graph)."""
        from ....core import in_capture_warmup

        if self.__dict__.get("_eig_ring") is None:
            # allocated by the eager step or the capture's warm-up, never inside a capture
            # (no host allocation while capturing; a counter zeroed inside the graph would be
            # reset by every replay)
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("CMAES: the eigensolver report ring must exist before a graph capture")
            self._eig_ring = torch.full((self.ESC_RING, 5), -1.0, dtype=torch.float64).pin_memory()
            self._eig_seq = torch.zeros(1, dtype=torch.int32, device=device)
        if in_capture_warmup():
            return None
        return self._eig_seq, self._eig_ring

    def _poll_eig_health(self, sc) -> None:
        target = sc["enqueued"] - self.ESC_LAG
        if target < 0 or target <= sc["checked"]:
            return
        sc["checked"] = target
        pend = sc["pending"]
        while pend and pend[0][0] < target:
            pend.popleft()
        if not pend or pend[0][0] != target:
            return
        _, ev, lvl = pend[0]
        ev.synchronize()  # the step two back: the GPU still holds the one after it
        row = self._eig_ring[target % self.ESC_RING].tolist()
        if int(row[4]) != target:
            return
        iters, capped = int(row[2]), bool((int(row[1]) & 1) or row[3])
        sc["history"].append((target, lvl, iters, capped))
        del sc["history"][:-64]
        level = sc["level"]
        if capped or iters >= self._level_slots(lvl):
            up = min(lvl + 1, self.TOP)
            if capped:
                sc["escalations"] += 1
        elif iters >= self._level_slots(level):
            up = lvl
        else:
            up = level
        if up > level:
            sc["level"], sc["streak"] = up, 0
            return
        if lvl == level and level > 0:
            fits = iters <= self._level_slots(level - 1) - 1
            sc["streak"] = sc["streak"] + 1 if fits else 0
            if sc["streak"] >= self.DOWN_STREAK:
                sc["level"], sc["streak"] = level - 1, 0

    @property
    def schedule_escalations(self) -> int:
        return int(self._sched()["escalations"])

    def schedule_levels(self, last: int = None) -> str:
        """The schedule each recent step replayed: L (late), V (warm, one slot fewer), W (warm), C (cold)."""
        lv = self._sched()["levels"]
        lv = lv if last is None else lv[-int(last):]
        return "".join("LVWC"[v] for v in lv)

    def graph_variant_context(self, variant):
        """The eigensolver schedule of a graph variant (ops/sbr_device.py: ``schedule``): "cold"
        — every slot full, bounds-gated damping; None — the warm schedule (lean tail slots);
        "late" — settled solves: damping / Newton–Schulz / order-6 kernels in the first slots only."""
        if variant in ("cold", "late", "warm6"):
            from ....ops.sbr_device import use_schedule

            return use_schedule(variant)
        return super().graph_variant_context(variant)

    # ------------------------------------------------------------------ sampling
    def _sample(self, state, key, row0: int, rows: int):
        d = self.dim
        if (state.B.is_cuda and d % 4 == 0 and config.get("gemm_prec") == "x6"
                and linalg.tall_nt_ok(rows, d, d, state.B.device)):
            # tall sampling product on the f16x3 LDS-staged GEMM: the Philox noise is generated
            # straight into its split planes (the f32 Z is never written), B·diag(D) split once
            # per generation with D as the column scale, σ and the mean in the epilogue
            za = linalg.normal_h3_planes(key.to(state.B.device), rows, d, row0)
            buf = state.population
            out = buf if (rows == self.pop_size and torch.cuda.is_current_stream_capturing() and buf.is_contiguous()
                          and buf.shape == (rows, d)) else None
            return linalg.tall_nt(za, state.B, alpha_ptr=state.sigma.reshape(1), bias_n=state.mean, b_colscale=state.D,
                                  out=out)
        z = rnd.normal(key, (rows, d), offset=row0 * d)
        if z.is_cuda:
            # X = mean + σ (Z∘D) Bᵀ = mean + Z (σ·B∘D)ᵀ : σ (a device scalar, no host sync)
            # folds into the d×d factor, leaving one plain GEMM with a bias epilogue
            if config.get("plain_gemm") == "blas":
                return plain_nt(z, (state.B * (state.D * state.sigma)).contiguous(), bias_n=state.mean)
            BD = (state.B * state.D).contiguous()
            buf = state.population
            if (rows == self.pop_size and torch.cuda.is_current_stream_capturing() and buf.is_contiguous()
                    and buf.shape == (rows, d)):
                # hipGraph: sample straight into the captured population buffer (the previous
                # generation's rows are dead once ask runs), so the state write-back has no 40 MB copy
                return mm(z, BD, tb=True, alpha_ptr=state.sigma.reshape(1), bias_n=state.mean, out=buf)
            return mm(z, BD, tb=True, alpha_ptr=state.sigma.reshape(1), bias_n=state.mean)
        return state.mean + state.sigma * (state.D * z) @ state.B.T

    def _counts_in_tell(self, state) -> bool:
        """The fused device tell advances count_iter (and count_eigen) inside its paths kernel —
        two one-element launches fewer per generation; ask then leaves count_iter as it is (the
        tell uses count_iter + 1, as the reference's ask would have set it)."""
        return self._fused_epilogue_ok(state)

    def _advance(self, state):
        return state if self._counts_in_tell(state) else state.update(count_iter=state.count_iter + 1)

    def ask(self, state):
        key, sample_key = rnd.split(state.key)
        population = self._sample(state, sample_key, 0, self.pop_size)
        return population, self._advance(state).update(population=population, key=key)

    # ------------------------------------------------------------------ tell
    def _aug_ok(self, population) -> bool:
        return population.is_cuda and config.get("plain_gemm") == "evoxmi"

    def _weighted_stats_aug(self, state, population, rows_i32, wvec):
        """The (d+1) × (d+1) rank-μ product of the centred, weighted rows augmented by a column
        σ·sqrt(wᵢ): its leading d × d block is Σ wᵢ yᵢ yᵢᵀ and its last row Σ wᵢ (xᵢ − m), the
        weighted mean shift — one centring pass and one GEMM instead of a weighted row sum (two
        launches) beside them (the (d+1)-wide product has the same tile grid as the d-wide one at
        d = 1000).  A view into a (d+1) × ld buffer (16-B rows)."""
        from ....ops import _ext

        d = self.dim
        Yw = _ext.ops().cma_center_rows(population, rows_i32, state.mean.contiguous(), state.sigma.reshape(1), wvec.contiguous(), True)
        ld = (d + 1 + 3) // 4 * 4
        S_aug = torch.empty(d + 1, ld, dtype=torch.float32, device=population.device)[:, : d + 1]
        return mm(Yw, Yw, ta=True, mode=1, out=S_aug)

    def _weighted_stats(self, state, population, order_i32, K: int, wvec, gather: bool, s_out=None):
        """(Σ wᵢ(xᵢ − m), Σ wᵢ yᵢ yᵢᵀ) with yᵢ = (xᵢ − m)/σ; ``s_out``: a (d, d) buffer the
        framework GEMM writes S into (the sharded tell's all-reduce buffer)."""
        d = self.dim
        if population.is_cuda:
            rows = order_i32 if gather else None
            one_over = state.sigma.reshape(1)
            # weighted mean shift: gathered weighted row sum (reduce.hip), deterministic
            dm = weighted_rowsum(population, rows, wvec, state.mean, K)
            if config.get("plain_gemm") in ("blas", "evoxmi"):
                # materialise Y = (x_sel − m)/σ once (K×d, 20 MB at the north-star shape) and
                # run the rank-μ product Yᵀ·(w∘Y) as one GEMM (weights are positive:
                # Σ wᵢ yᵢ yᵢᵀ = Ywᵀ Yw with Yw = y·sqrt(w), one fused gather/centre/scale pass,
                # cmaes.hip); the framework GEMM computes only the upper tiles of the
                # symmetric product
                from ....ops import _ext

                Yw = _ext.ops().cma_center_rows(population, rows, state.mean.contiguous(), state.sigma.reshape(1),
                                                wvec.contiguous())
                if config.get("plain_gemm") == "blas":
                    return dm, torch.mm(Yw.t(), Yw)
                return dm, mm(Yw, Yw, ta=True, mode=1, out=s_out)
            splits = max(1, min(16, K // 256))
            S = gemm(
                Operand(population, rc=True, gather=rows, sub=state.mean, kw=wvec, sscale=one_over, sscale_inv=True),
                Operand(population, rc=True, gather=rows, sub=state.mean, sscale=one_over, sscale_inv=True),
                d, d, K, splits=splits,
            )
            S = S.sum(0) if S.dim() == 3 else S
            return dm, S
        sel = population[order_i32.long()] if gather else population
        diff = sel - state.mean
        dm = wvec @ diff
        y = diff / state.sigma
        S = (y.T * wvec) @ y
        return dm, S

    def _fused_epilogue_ok(self, state):
        return (state.C.is_cuda and self.decomp_per_iter == 1 and config.get("cma_fused")
                and config.get("eigh") in ("jacobi", "sbr") and state.count_iter.dtype == torch.int64)

    def _finish_tell_fused(self, state, dm, S):
        """Same update as ``_finish_tell`` in four fused kernels around the eigensolver
        (``cmaes.hip``): δ/invsqrtC·δ, the evolution paths and σ, the covariance blend
        with the padded eigensolver operands, and the eigenbasis extraction."""
        from ....ops import _ext, jacobi

        ops = _ext.ops()
        d = self.dim
        mean, delta, y = ops.cma_delta_gemv(state.invsqrtC.contiguous(), state.mean.contiguous(), dm.contiguous(), float(self.cm))
        consts = [self.cs, math.sqrt(self.cs * (2 - self.cs) * self.mueff), self.cc, math.sqrt(self.cc * (2 - self.cc) * self.mueff),
                  self.chiN, self.damps, self.c1, self.cmu, (1.4 + 2 / (d + 1)) * self.chiN]
        ps, pc, sigma, a, _hsig, count_iter, count_eigen = ops.cma_paths(
            state.ps.contiguous(), state.pc.contiguous(), y, delta, state.sigma.reshape(1).contiguous(), state.count_iter.reshape(1).contiguous(),
            consts, state.count_eigen.reshape(1).contiguous())
        eig_stats = state.eig_stats
        # hipGraph: C' and B go straight into the captured state buffers (no write-back copy of
        # 8 MB per generation): cov_pad reads each C element only where it writes it, and the
        # old B is last read by the eigensolver, before cma_eig_out
        capturing = torch.cuda.is_current_stream_capturing()
        c_out = state.C if capturing and state.C.is_contiguous() else None
        b_out = state.B if capturing and state.B.is_contiguous() else None
        if config.get("eigh") == "sbr":
            np_ = jacobi.padded_size(d)
            C, Cp, _ = ops.cma_cov_pad(state.C.contiguous(), S if S.stride(1) == 1 else S.contiguous(), pc, a, float(self.c1),
                                       float(self.cmu), state.B.contiguous(), np_, c_out, False)
            # Cp[:d, :d] = triu(C) + triu(C, 1)ᵀ, the reference's symmetrisation (cma_es.py:193-195)
            with profiling.phase("eigh"):
                if config.get("sbr_mode") == "device" and d % 4 == 0 and d <= 8192:
                    # converged solve as a fixed device-controlled schedule: part of the
                    # generation's graph, no host read (ops/sbr_device.py)
                    from ....ops.sbr_device import eigh_device

                    # restore=False: a diverged solve's warm start is selected by cma_eig_out itself
                    # (keep word), not copied back by a launch of its own
                    w, Bn, eig_stats, keep = eigh_device(Cp[:d, :d], state.B, report=self._report_buffers(state.B.device),
                                                         restore=False)
                else:
                    # host-orchestrated solve: a host phase between hipGraph segments
                    w, Bn, eig_stats = host_phase(sbr_phase, Cp[:d, :d], state.B, self.__dict__.setdefault("_eig_plans", {}),
                                                  out_like=(state.D, state.B, state.eig_stats))
                    keep = None
            B, D, BdivD = ops.cma_eig_out(Bn.contiguous(), w.contiguous(), d, b_out, state.B.contiguous() if keep is not None else None,
                                          keep)
        else:
            np_ = jacobi.padded_size(d)
            C, Cp, Bp = ops.cma_cov_pad(state.C.contiguous(), S if S.stride(1) == 1 else S.contiguous(), pc, a, float(self.c1),
                                        float(self.cmu), state.B.contiguous(), np_,
                                        c_out, True)
            with profiling.phase("eigh"):
                w, Bp = jacobi.warm_eigh_padded(Cp, Bp, d, max_sweeps=self.eig_sweeps)
            B, D, BdivD = ops.cma_eig_out(Bp, w, d, b_out)
        # (B/D)·Bᵀ is symmetric: upper tiles only
        if config.get("plain_gemm") == "blas":
            invsqrtC = plain_nt(BdivD, B)
        elif capturing and state.invsqrtC.is_contiguous():
            # hipGraph: the old invsqrtC was last read by cma_delta_gemv above (stream order), so the
            # new one goes straight into the captured buffer
            invsqrtC = mm(BdivD, B, tb=True, mode=1, out=state.invsqrtC)
        else:
            invsqrtC = mm(BdivD, B, tb=True, mode=1)
        # outside a graph the stats buffer is the solver's own and is reused: the state keeps a copy
        # (under capture the state write-back is that copy)
        return state.update(mean=mean, ps=ps, pc=pc, C=C, sigma=sigma.reshape(state.sigma.shape), B=B, D=D, invsqrtC=invsqrtC,
                            count_iter=count_iter.reshape(state.count_iter.shape), count_eigen=count_eigen.reshape(state.count_eigen.shape),
                            eig_stats=eig_stats if capturing else eig_stats.clone())

    def _finish_tell(self, state, dm, S):
        if self._fused_epilogue_ok(state):
            return self._finish_tell_fused(state, dm, S)
        d = self.dim
        mean = state.mean + self.cm * dm
        delta_mean = mean - state.mean
        ps = (1 - self.cs) * state.ps + math.sqrt(self.cs * (2 - self.cs) * self.mueff) * (state.invsqrtC @ delta_mean) / state.sigma
        count = state.count_iter.to(torch.float32)
        hsig = (torch.linalg.norm(ps) / torch.sqrt(1 - (1 - self.cs) ** (2 * count)) < (1.4 + 2 / (d + 1)) * self.chiN).to(torch.float32)
        pc = (1 - self.cc) * state.pc + hsig * math.sqrt(self.cc * (2 - self.cc) * self.mueff) * delta_mean / state.sigma
        a = (1 - self.c1 - self.cmu) + self.c1 * (1 - hsig) * self.cc * (2 - self.cc)
        C = a * state.C + self.c1 * torch.outer(pc, pc) + self.cmu * S
        sigma = state.sigma * torch.exp((self.cs / self.damps) * (torch.linalg.norm(ps) / self.chiN - 1))
        B, D, invsqrtC, count_eigen = self._maybe_decompose(state, C)
        return state.update(mean=mean, ps=ps, pc=pc, C=C, sigma=sigma, B=B, D=D, invsqrtC=invsqrtC, count_eigen=count_eigen)

    def _maybe_decompose(self, state, C):
        if self.decomp_per_iter > 1 and int(state.count_iter) % self.decomp_per_iter != 0:
            return state.B, state.D, state.invsqrtC, state.count_eigen
        return (*self._decomposition_C(C, state.B), state.count_eigen + 1)

    def _decomposition_C(self, C, B_prev):
        Cs = symmetrize_upper(C)
        d = self.dim
        if (Cs.is_cuda and config.get("eigh") == "sbr" and config.get("sbr_mode") == "device" and d % 4 == 0 and d <= 8192
                and self.eig_sweeps is None):
            # decompositions every decomp_per_iter generations (small λ): the matrix moved by several
            # updates since the last basis, so the device solver runs the cold-start rules (every slot
            # full, bounds-gated damping) with twice the cold slots ("deep"): the host driver's plain
            # refinement fell back to Jacobi sweeps in 25 of 28 such solves at d = 1000, λ = 24, and
            # with the 16 cold slots 5 of 25 solves that recovered from a divergence were capped
            # (damped steps after a recovery converge slowly; profiles/NOTES.md, round 6)
            from ....ops.sbr_device import eigh_device, use_schedule

            with use_schedule("deep"):
                w, B, _ = eigh_device(Cs.contiguous(), B_prev.contiguous())
            w, B = w.clone(), B.clone()
        else:
            w, B = warm_eigh(Cs, B_prev, max_sweeps=self.eig_sweeps, plans=self.__dict__.setdefault("_eig_plans", {}))
        B = B.contiguous()
        w = torch.clamp(w, min=1e-30)
        D = torch.sqrt(w)
        if B.is_cuda:
            invsqrtC = plain_nt(B / D, B) if config.get("plain_gemm") == "blas" else mm((B / D).contiguous(), B, tb=True, mode=1)
        else:
            invsqrtC = (B / D) @ B.T
        return B, D, invsqrtC

    def tell(self, state, fitness):
        pop = state.population
        if self._aug_ok(pop):
            _, order = argsort_i32(fitness.contiguous())
            S_aug = self._weighted_stats_aug(state, pop, order[: self.mu].contiguous(), self.weights)
            d = self.dim
            dm, S = S_aug[d, :d], S_aug[:d, :d]
        elif pop.is_cuda:
            _, order = argsort_i32(fitness.contiguous())
            dm, S = self._weighted_stats(state, pop, order[: self.mu].contiguous(), self.mu, self.weights, gather=True)
        else:
            _, order = argsort(fitness)
            dm, S = self._weighted_stats(state, pop, order[: self.mu], self.mu, self.weights, gather=True)
        return self._finish_tell(state, dm, S)

    # ------------------------------------------------------------------ SPMD protocol
    def ask_sharded(self, state, dist):
        start, size = dist.slice_of(self.pop_size)
        key, sample_key = rnd.split(state.key)
        local = self._sample(state, sample_key, start, size)
        return local, self._advance(state).update(population=local, key=key)

    def tell_sharded(self, state, fitness, dist):
        """``fitness`` is the all-gathered (λ,) vector; ``state.population`` the local rows.

        One global argsort; this rank's rows among the top μ are compacted in global-rank order
        by one kernel (``cma_local_select``: at most K = min(μ, λ/N) of them — the same K = μ
        GEMM as the unsharded tell on one rank, static for hipGraphs, padded with zero weights);
        the rank-μ partial sum S (symmetric) goes on the wire as its packed upper triangle with
        the weighted mean shift appended: d(d+1)/2 + d floats, half the bytes of round 5's
        (d² + d) all-reduce.  Reference: ``cma_es.py:163-198`` (tell), whose ``Σ wᵢ yᵢ yᵢᵀ`` is
        this sum over ranks."""
        start, size = dist.slice_of(self.pop_size)
        d = self.dim
        K = min(self.mu, size)
        dev = fitness.device
        if fitness.is_cuda:
            from ....ops import _ext

            ops = _ext.ops()
            _, order = argsort_i32(fitness.contiguous())
            lsel = torch.empty(K, dtype=torch.int32, device=dev)
            wsel = torch.empty(K, dtype=torch.float32, device=dev)
            ops.cma_local_select(order, self.mu, self.weights, start, size, lsel, wsel)
        else:
            _, order = argsort(fitness)
            top = order[: self.mu]
            mine = (top >= start) & (top < start + size)
            lsel = torch.zeros(K, dtype=torch.int64)
            wsel = torch.zeros(K, dtype=torch.float32)
            n = int(mine.sum())
            lsel[:n] = top[mine] - start
            wsel[:n] = self.weights.cpu()[mine]
            lsel, wsel = lsel.to(dev), wsel.to(dev)
        if self._aug_ok(state.population):
            # the augmented product's packed upper triangle carries the mean shift in its last
            # column: (d+1)(d+2)/2 floats on the wire, one more than d(d+1)/2 + d
            from ....ops import _ext

            ops = _ext.ops()
            S_aug = self._weighted_stats_aug(state, state.population, lsel, wsel)
            Pa = (d + 1) * (d + 2) // 2
            buf = torch.empty(Pa, dtype=torch.float32, device=dev)
            ops.sym_pack(S_aug, buf)
            with profiling.phase("all_reduce"):
                dist.all_reduce_(buf)
            ops.sym_unpack(buf, S_aug)
            return self._finish_tell(state, S_aug[d, :d], S_aug[:d, :d])
        dm, S = self._weighted_stats(state, state.population, lsel, K, wsel, gather=True)
        P = d * (d + 1) // 2
        buf = torch.empty(P + d, dtype=torch.float32, device=dev)
        if S.is_cuda:
            ops.sym_pack(S, buf[:P])
        else:
            iu = torch.triu_indices(d, d)
            buf[:P] = S[iu[0], iu[1]]
        buf[P:].copy_(dm.reshape(-1))
        with profiling.phase("all_reduce"):
            dist.all_reduce_(buf)
        if S.is_cuda:
            ops.sym_unpack(buf[:P], S)
        else:
            S = torch.zeros(d, d, dtype=torch.float32)
            S[iu[0], iu[1]] = buf[:P]
            S = S + torch.triu(S, 1).T
        return self._finish_tell(state, buf[P:], S)


class SepCMAES(ColumnSeparable, CMAES):
    """Separable CMA-ES (diagonal covariance, linear time/space).

    Decision-axis state sharding (P2): mean, paths, diag(C) and the population are column
    blocks; the noise is drawn per global column (normal_cols) and the one cross-column
    quantity, ‖p_σ‖, is an all-reduced sum of squares (col_sum) — the collective GSPMD
    inserts for the same norm over a sharded axis."""

    column_separable = True
    dim_fields = ("pc", "ps", "C", "mean", "population")

    # no eigensolver: one graph, no schedule variants (ADVICE r5 — the inherited ones captured
    # three identical graphs)
    def _device_eigh(self) -> bool:
        return False

    def graph_variant(self, generation: int):
        return None

    def graph_variant_set(self):
        return ()

    def setup(self, key):
        dev = self.center_init.device
        d = self.dim
        return State(
            pc=torch.zeros(d, device=dev),
            ps=torch.zeros(d, device=dev),
            C=torch.ones(d, device=dev),
            count_iter=torch.zeros((), dtype=torch.int64, device=dev),
            mean=self.center_init.to(torch.float32).clone(),
            sigma=torch.tensor(self.init_stdev, dtype=torch.float32, device=dev),
            key=key.to(dev),
            population=torch.zeros((self.pop_size, d), device=dev),
            # last decomposition: [relative off-norm, Jacobi sweeps, refinement iterations, fallback]
            eig_stats=torch.zeros(4, dtype=torch.float64, device=dev),
        )

    def ask(self, state):
        key, sample_key = rnd.split(state.key)
        noise = self.normal_cols(sample_key, self.pop_size, state.mean.device)
        population = state.mean + state.sigma * torch.sqrt(state.C) * noise
        return population, state.update(population=population, count_iter=state.count_iter + 1, key=key)

    def tell(self, state, fitness):
        _, order = argsort(fitness)
        sel = state.population[order[: self.mu]]
        mean = state.mean + self.cm * (self.weights @ (sel - state.mean))
        delta_mean = mean - state.mean
        ps = (1 - self.cs) * state.ps + math.sqrt(self.cs * (2 - self.cs) * self.mueff) * delta_mean / torch.sqrt(state.C) / state.sigma
        count = state.count_iter.to(torch.float32)
        ps_norm = torch.sqrt(self.col_sum((ps * ps).sum()))
        hsig = (ps_norm / torch.sqrt(1 - (1 - self.cs) ** (2 * count)) < (1.4 + 2 / (self.dim + 1)) * self.chiN).to(torch.float32)
        pc = (1 - self.cc) * state.pc + hsig * math.sqrt(self.cc * (2 - self.cc) * self.mueff) * delta_mean / state.sigma
        y = (sel - state.mean) / state.sigma
        C = (1 - self.c1 - self.cmu) * state.C + self.c1 * (pc**2 + (1 - hsig) * self.cc * (2 - self.cc) * state.C) + self.cmu * (self.weights @ (y**2))
        sigma = state.sigma * torch.exp((self.cs / self.damps) * (ps_norm / self.chiN - 1))
        return state.update(mean=mean, ps=ps, pc=pc, C=C, sigma=sigma)


class IPOPCMAES(CMAES):
    """Restart CMA-ES with increasing population (Auger & Hansen 2005).

    The reference version cannot change its (static) sample count and uses a
    removed ``lax.cond`` signature.  Here restarts are real:
    on stagnation for ``stagnation_threshold`` generations the distribution is
    reset (mean = ``center_init``, σ = ``init_stdev``, C = I) and λ doubles; the
    recombination weights and learning rates are recomputed for the new λ.
    Host-side control flow ⇒ not graph-capturable.
    """

    def __init__(self, center_init, init_stdev, pop_size=None, recombination_weights=None, cm=1, stagnation_threshold=50, max_pop_size=None):
        super().__init__(center_init, init_stdev, pop_size, recombination_weights, cm)
        self.original_pop_size = self.pop_size
        self.stagnation_threshold = stagnation_threshold
        self.max_pop_size = max_pop_size

    def setup(self, key):
        st = super().setup(key)
        return st.update(best_fitness=float("inf"), restarts=0, stagnation_count=0, pop_size=self.pop_size)

    def _configure(self, pop_size):
        self.pop_size = pop_size
        self.mu = pop_size // 2
        self.weights = _default_weights(self.mu).to(self.center_init.device)
        self._set_rates()

    def ask(self, state):
        if state.pop_size != self.pop_size:
            self._configure(state.pop_size)
        return super().ask(state)

    def _next_pop_size(self, state):
        return self.original_pop_size * (2 ** (state.restarts + 1))

    def tell(self, state, fitness):
        state = super().tell(state, fitness)
        cur = float(fitness.min())
        if cur < state.best_fitness:
            state = state.update(best_fitness=cur, stagnation_count=0)
        else:
            state = state.update(stagnation_count=state.stagnation_count + 1)
        if state.stagnation_count >= self.stagnation_threshold:
            new_pop = self._next_pop_size(state)
            if self.max_pop_size is not None:
                new_pop = min(new_pop, self.max_pop_size)
            d, dev = self.dim, self.center_init.device
            state = state.update(
                restarts=state.restarts + 1,
                pop_size=new_pop,
                stagnation_count=0,
                best_fitness=float("inf"),
                sigma=torch.tensor(self.init_stdev, dtype=torch.float32, device=dev),
                mean=self.center_init.to(torch.float32).clone(),
                C=torch.eye(d, device=dev),
                B=torch.eye(d, device=dev),
                D=torch.ones(d, device=dev),
                invsqrtC=torch.eye(d, device=dev),
                pc=torch.zeros(d, device=dev),
                ps=torch.zeros(d, device=dev),
                count_iter=torch.zeros((), dtype=torch.int64, device=dev),
            )
        return state


class BIPOPCMAES(IPOPCMAES):
    """Bi-population restarts: large-population regime doubles λ; once λ exceeds
    16× the original it falls back to the original size (reference ``:359-390``)."""

    def _next_pop_size(self, state):
        if state.pop_size > 16 * self.original_pop_size:
            return self.original_pop_size
        return state.pop_size * 2
