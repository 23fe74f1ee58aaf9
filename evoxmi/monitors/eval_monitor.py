"""Evaluation monitor (reference ``src/evox/monitors/eval_monitor.py:16-215``).

Same public API (``get_best_fitness``, ``get_topk_solutions``, ``get_pf_fitness``,
``get_history``, ``plot``, ``flush`` ...).  MI355X-first execution: the reference
ships top-k rows to the host through ``io_callback`` every generation; here the
top-k merge (SO) and the Pareto archive (MO) stay **device resident** and are
computed with stream-ordered device ops only — ``post_eval`` never synchronises
the host with the GPU, so it does not stall the generation pipeline (and works
with graph replay, which hands it the graph's static output buffers).  Host
copies happen only when a getter is called.
"""
from __future__ import annotations

import warnings

import torch
import torch.utils._pytree as pytree

from ..core import Monitor
from .async_d2h import D2HCopier, HostList


def _apply_dir(x, od):
    if isinstance(od, torch.Tensor):
        return x * od.to(x.device)
    return x if od == 1 else x * od


def _check_kernels():
    from ..ops import _ext

    if _ext._ERR:
        _ext.check_kernel_errors()


class EvalMonitor(Monitor):
    def __init__(self, full_fit_history=True, full_sol_history=False, topk=1, calc_pf=False, history_to_host=False):
        super().__init__()
        self.full_fit_history = full_fit_history
        self.full_sol_history = full_sol_history
        self.topk = topk
        self.calc_pf = calc_pf
        self.history_to_host = history_to_host
        # history_to_host: entries are copied to pinned host memory on a side stream
        # (async_d2h.D2HCopier) and resolved when read
        self.fitness_history = HostList()
        self.solution_history = HostList()
        self._d2h = D2HCopier() if history_to_host else None
        self.topk_fitness = None
        self.topk_solutions = None
        self.pf_solutions = None
        self.pf_fitness = None
        self.latest_solution = None
        self.latest_fitness = None
        self.eval_count = 0
        self.opt_direction = 1
        self._dist = None

    def hooks(self):
        return ["post_eval"]

    def set_opt_direction(self, opt_direction):
        self.opt_direction = opt_direction

    def set_dist(self, ctx):
        """Population-sharded runs: candidate rows are rank-local (the workflow's
        ``enable_distributed``).  The best solution is then found with ONE MINLOC
        all-reduce over the ranks' local minima (packed ordered-f32 | global index,
        ``DistContext.all_reduce_min_loc``) and its row assembled by a SUM all-reduce
        to which only the owner contributes (graph-safe: no host-side owner lookup)."""
        self._dist = ctx

    def _sharded_best(self, local_sol, fitness):
        d = self._dist
        n = fitness.shape[0]
        start, size = d.slice_of(n)
        f_loc = fitness[start : start + size]
        i_loc = torch.argmin(f_loc)
        val, gidx = d.all_reduce_min_loc(f_loc[i_loc], i_loc + start)
        mine = gidx == i_loc + start
        row = local_sol.index_select(0, i_loc.reshape(1))
        # select, not multiply: a non-owner's inf/NaN row times 0 would poison the sum
        row = torch.where(mine, row, torch.zeros_like(row))
        d.all_reduce_(row)
        return val.reshape(1), row

    def _keep(self, x):
        if x is None:
            return None
        if self._d2h is not None and isinstance(x, torch.Tensor):
            return self._d2h.submit(x)
        return pytree.tree_map(lambda t: t.detach().clone() if isinstance(t, torch.Tensor) else t, x)

    def post_eval(self, _state, cand_sol, _transformed, fitness):
        self.eval_count += int(fitness.shape[0])
        if fitness.ndim == 1:
            self.record_fit_single_obj(cand_sol, fitness)
        else:
            self.record_fit_multi_obj(cand_sol, fitness)

    # candidate solutions may be tensors or pytrees of tensors (e.g. TreeAlgorithm,
    # neuroevolution parameter trees): every row operation is applied leaf-wise
    @staticmethod
    def _rows(sol):
        leaves = [x for x in pytree.tree_leaves(sol) if isinstance(x, torch.Tensor)]
        return leaves[0].shape[0] if leaves else None

    @staticmethod
    def _sel(sol, idx):
        return pytree.tree_map(lambda x: x.index_select(0, idx) if isinstance(x, torch.Tensor) else x, sol)

    @staticmethod
    def _where(better, a, b):
        return pytree.tree_map(lambda x, y: torch.where(better.reshape((-1,) + (1,) * (x.dim() - 1)), x, y), a, b)

    @staticmethod
    def _cat(a, b):
        return pytree.tree_map(lambda x, y: torch.cat([x, y], 0), a, b)

    @staticmethod
    def _clone(a):
        return pytree.tree_map(lambda x: x.clone() if isinstance(x, torch.Tensor) else x, a)

    def record_fit_single_obj(self, cand_sol, fitness):
        if self.full_sol_history:
            self.solution_history.append(self._keep(cand_sol))
        if self.full_fit_history:
            self.fitness_history.append(self._keep(fitness))
        n = fitness.shape[0]
        k = min(self.topk, n)
        if cand_sol is not None and self._rows(cand_sol) != n:
            if k == 1 and self._dist is not None and isinstance(cand_sol, torch.Tensor):
                fit, sol = self._sharded_best(cand_sol, fitness)
                if self.topk_fitness is None:
                    self.topk_fitness, self.topk_solutions = fit.clone(), sol.clone()
                else:
                    better = fit < self.topk_fitness
                    self.topk_fitness = torch.where(better, fit, self.topk_fitness)
                    self.topk_solutions = torch.where(better[:, None], sol, self.topk_solutions)
                return
            cand_sol = None  # rows are sharded and there is no context: fitness only
        if k == 1:
            i = torch.argmin(fitness)
            fit = fitness.index_select(0, i.reshape(1))
            sol = self._sel(cand_sol, i.reshape(1)) if cand_sol is not None else None
            if self.topk_fitness is None:
                self.topk_fitness, self.topk_solutions = fit.clone(), (self._clone(sol) if sol is not None else None)
            else:
                better = fit < self.topk_fitness  # device-side select, no host sync
                self.topk_fitness = torch.where(better, fit, self.topk_fitness)
                if sol is not None and self.topk_solutions is not None:
                    self.topk_solutions = self._where(better, sol, self.topk_solutions)
        else:
            vals, idx = torch.topk(fitness, k, largest=False, sorted=True)
            sols = self._sel(cand_sol, idx) if cand_sol is not None else None
            if self.topk_fitness is not None:
                vals = torch.cat([self.topk_fitness, vals])
                if sols is not None and self.topk_solutions is not None:
                    sols = self._cat(self.topk_solutions, sols)
                v2, i2 = torch.topk(vals, k, largest=False, sorted=True)
                vals = v2
                if sols is not None:
                    sols = self._sel(sols, i2)
            self.topk_fitness, self.topk_solutions = vals, sols

    def record_fit_multi_obj(self, cand_sol, fitness):
        from ..operators.selection.non_dominate import non_dominated_sort

        if self.full_sol_history:
            self.solution_history.append(self._keep(cand_sol))
        if self.full_fit_history:
            self.fitness_history.append(self._keep(fitness))
        if self.calc_pf:
            pf_f = fitness if self.pf_fitness is None else torch.cat([self.pf_fitness, fitness], 0)
            pf_s = cand_sol if self.pf_solutions is None else torch.cat([self.pf_solutions, cand_sol], 0)
            rank = non_dominated_sort(pf_f)
            keep = rank == 0
            self.pf_fitness = pf_f[keep]
            self.pf_solutions = pf_s[keep]
        self.latest_fitness = fitness.detach().clone()
        self.latest_solution = cand_sol.detach().clone() if cand_sol is not None else None

    # ---------------------------------------------------------------- getters
    # Getters are host sync points: a kernel failure recorded in the sticky device error
    # word (e.g. the NDS grid barrier timing out) raises here instead of going unnoticed.
    def get_latest_fitness(self):
        _check_kernels()
        return _apply_dir(self.latest_fitness, self.opt_direction)

    def get_latest_solution(self):
        return self.latest_solution

    def get_pf_fitness(self):
        _check_kernels()
        return _apply_dir(self.pf_fitness, self.opt_direction)

    def get_pf_solutions(self):
        return self.pf_solutions

    def get_topk_fitness(self):
        _check_kernels()
        return _apply_dir(self.topk_fitness, self.opt_direction)

    def get_topk_solutions(self):
        return self.topk_solutions

    def get_best_solution(self):
        return None if self.topk_solutions is None else self.topk_solutions[0]

    def get_best_fitness(self):
        _check_kernels()
        if self.topk_fitness is None:
            warnings.warn("trying to get info from a monitor with no recorded data")
            return None
        return _apply_dir(self.topk_fitness[0], self.opt_direction)

    def get_history(self):
        return [_apply_dir(f, self.opt_direction) for f in self.fitness_history]

    def plot(self, problem_pf=None, **kwargs):
        from ..vis_tools import plot

        if not self.fitness_history:
            warnings.warn("No fitness history recorded, return None")
            return None
        h = [f.cpu() for f in self.get_history()]
        n_objs = 1 if h[0].ndim == 1 else h[0].shape[1]
        if n_objs == 1:
            return plot.plot_obj_space_1d(h, **kwargs)
        if n_objs == 2:
            return plot.plot_obj_space_2d(h, problem_pf, **kwargs)
        if n_objs == 3:
            return plot.plot_obj_space_3d(h, problem_pf, **kwargs)
        warnings.warn("Not supported yet.")
        return None

    def flush(self):
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        _check_kernels()

    def close(self):
        self.flush()
