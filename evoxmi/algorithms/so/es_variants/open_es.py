"""OpenES (Salimans et al. 2017; reference ``es_variants/open_es.py:19-82``).

Mirrored sampling ``ε, −ε``, gradient ``εᵀ f / (N σ)``, plain SGD step or an optimiser
sub-module (``optimizer='adam'``).  The noise matrix is never stored: ``ask``
keeps only its Philox key, and ``tell`` regenerates ε(i, j) inside the gradient kernel
(``rng.hip: es_noise_grad_kernel``, one fused pass; mirrored pairs folded into the
weights ``f_i − f_{i+N/2}``).  At pop 8192 × 6 k parameters that drops a 200 MB buffer.

SPMD protocol (north-star config 4, population sharded over the GPUs of a node):
``ask_sharded`` generates only this rank's rows of the (virtual, mirrored) noise matrix
from the Philox counters — row ``g`` is ``half[g]`` or ``−half[g − N/2]`` exactly as in
``ask`` — and ``tell_sharded`` regenerates the same rows inside the gradient kernel and
all-reduces the rank's partial gradient (P floats) over RCCL; the centre/optimiser state
stays replicated and bit-identical on every rank.
"""
from __future__ import annotations

import torch

from ....core import Algorithm, State, use_state
from ....ops import _ext
from ....ops import random as rnd
from ....parallel.dim_sharded import ColumnSeparable
from ._common import make_optimizer


def _normal_rows(key, rows: int, d: int, row0: int, dev):
    """Rows [row0, row0 + rows) of the virtual normal matrix normal(key, (·, d)).  On the
    device always through the Philox fill kernel (the same Box–Muller arithmetic as the
    gradient kernel's regeneration, bit for bit)."""
    if dev.type == "cuda":
        off = row0 * d
        lead = off & 3
        flat = _ext.philox_fill(key.to(dev).contiguous(), rows * d + lead, 1, off - lead)
        return flat[lead:].reshape(rows, d)
    return rnd.normal(key, (rows, d), offset=row0 * d).to(dev)


def _noise_grad(key, w, d: int, row0: int, dev, cols=None):
    """Σ_i w[i] · normal(key)[row0 + i, :] without materialising the rows on the device;
    ``cols = (col0, own)``: only the column window [col0, col0 + own) of the d columns."""
    c0, own = cols if cols is not None else (0, d)
    if w.numel() == 0:
        return torch.zeros(own, device=dev)
    if dev.type == "cuda":
        return _ext.ops().es_noise_grad(key.to(dev).contiguous(), w.to(torch.float32).contiguous(), int(own), int(row0), int(c0), int(d))
    if cols is not None:
        return rnd.normal_window(key, w.shape[0], d, c0, own, row0, dev).T @ w.to(torch.float32)
    return _normal_rows(key, w.shape[0], d, row0, dev).T @ w.to(torch.float32)


class OpenES(ColumnSeparable, Algorithm):
    rank_local_fields = ("population",)
    # decision-axis state sharding (StdWorkflow.enable_multi_devices(shard_state=True)): the
    # centre, the population and an element-wise optimiser's state are column blocks; every
    # rank draws only its columns of the (virtual) Philox noise (es_population / es_noise_grad
    # with a column window) and reduces εᵀf over them
    column_separable = True
    dim_fields = ("population", "center")
    dim_child_fields = {"optimizer": ("opt_state",)}

    def __init__(self, center_init, pop_size, learning_rate, noise_stdev, optimizer=None, mirrored_sampling=True):
        super().__init__()
        assert noise_stdev > 0 and learning_rate > 0 and pop_size > 0
        if mirrored_sampling:
            assert pop_size % 2 == 0, "When mirrored_sampling is True, pop_size must be a multiple of 2."
        self.dim = center_init.shape[0]
        self.center_init = center_init
        self.pop_size = pop_size
        self.learning_rate = learning_rate
        self.noise_stdev = noise_stdev
        self.mirrored_sampling = mirrored_sampling
        self.optimizer = make_optimizer(optimizer, learning_rate, center_init) if optimizer == "adam" else None
        self._opt_name = optimizer

    def setup(self, key):
        pop = self.center_init.expand(self.pop_size, -1).clone()
        return State(population=pop, center=self.center_init.clone(), noise_key=key.clone(), key=key)

    def dim_shard(self, state, col0: int, own: int):
        if self.optimizer is not None and getattr(self, "_opt_name", "adam") not in ("adam", "sgd"):
            raise ValueError("OpenES column sharding needs an element-wise optimiser (none, 'sgd' or 'adam')")
        if self.optimizer is None:
            self.dim_child_fields = {}
        return super().dim_shard(state, col0, own)

    def ask(self, state):
        key, noise_key = rnd.split(state.key)
        dev = state.center.device
        if self._cols is None:
            population = self._population_rows(noise_key, state.center, 0, self.pop_size)
        else:  # column block of a decision-axis-sharded state: only this rank's noise columns are drawn
            population = self._population_rows(noise_key, state.center, 0, self.pop_size, cols=self.cols())
        return population, state.update(population=population, key=key, noise_key=noise_key.to(state.noise_key.device))

    def _population_rows(self, noise_key, center, start: int, size: int, cols=None):
        """Rows [start, start + size) of center + σ·ε (mirrored: −ε for the second half).  On the
        device ONE kernel (rng.hip: es_population_kernel) draws the same Philox noise as
        :meth:`_noise_rows` and writes the rows; the noise matrix, its negated copy and their
        concatenation are never materialised."""
        c0, own, dtot = cols if cols is not None else (0, center.shape[0], center.shape[0])
        if center.is_cuda and center.dtype == torch.float32:
            half = self.pop_size // 2 if self.mirrored_sampling else 0
            return _ext.ops().es_population(noise_key.to(center.device).contiguous(), center.contiguous(), float(self.noise_stdev),
                                            int(size), int(half), int(start), int(c0), int(dtot))
        noise = self._noise_rows(noise_key, start, size, center.device)
        return center[None, :] + self.noise_stdev * (noise[:, c0 : c0 + own] if cols is not None else noise)

    def _grad_rows(self, noise_key, fitness, start: int, size: int, dev, cols=None):
        """Σ over global rows [start, start + size) of f_g ε_g (f indexed by global row);
        ``cols = (col0, own)``: only that column window of ε."""
        d = self.dim
        width = cols[1] if cols is not None else d
        f = fitness.to(torch.float32)
        if not self.mirrored_sampling:
            return _noise_grad(noise_key, f[start : start + size], d, start, dev, cols)
        h = self.pop_size // 2
        g = torch.zeros(width, device=dev)
        a0, a1 = start, min(start + size, h)
        b0, b1 = max(start, h), start + size
        if a1 > a0 and b0 == h and b1 - h == a1 - a0 and a0 == 0:
            # whole population on one rank: mirrored pairs folded into one pass
            return _noise_grad(noise_key, f[:h] - f[h:], d, 0, dev, cols)
        if a1 > a0:
            g = g + _noise_grad(noise_key, f[a0:a1], d, a0, dev, cols)
        if b1 > b0:
            g = g - _noise_grad(noise_key, f[b0:b1], d, b0 - h, dev, cols)
        return g

    def tell(self, state, fitness):
        cols = (self.cols()[0], self.cols()[1]) if self._cols is not None else None
        grad = self._grad_rows(state.noise_key, fitness, 0, self.pop_size, state.center.device, cols) / self.pop_size / self.noise_stdev
        if self.optimizer is None:
            center = state.center - self.learning_rate * grad
        else:
            updates, state = use_state(self.optimizer.update)(state, grad, state.center)
            center = state.center + updates
        return state.update(center=center)

    # ------------------------------------------------------------------ SPMD protocol
    def _noise_rows(self, key, start: int, size: int, dev):
        """Global rows [start, start + size) of the (mirrored) noise matrix."""
        d = self.dim
        if not self.mirrored_sampling:
            return _normal_rows(key, size, d, start, dev)
        h = self.pop_size // 2
        parts = []
        a0, a1 = start, min(start + size, h)
        if a1 > a0:
            parts.append(_normal_rows(key, a1 - a0, d, a0, dev))
        b0, b1 = max(start, h) - h, start + size - h
        if b1 > b0:
            parts.append(-_normal_rows(key, b1 - b0, d, b0, dev))
        return parts[0] if len(parts) == 1 else torch.cat(parts, 0)

    def ask_sharded(self, state, dist):
        start, size = dist.slice_of(self.pop_size)
        key, noise_key = rnd.split(state.key)
        population = self._population_rows(noise_key, state.center, start, size)
        return population, state.update(population=population, key=key, noise_key=noise_key.to(state.noise_key.device))

    def tell_sharded(self, state, fitness, dist):
        start, size = dist.slice_of(self.pop_size)
        g = self._grad_rows(state.noise_key, fitness, start, size, state.center.device)
        dist.all_reduce_(g)
        grad = g / self.pop_size / self.noise_stdev
        if self.optimizer is None:
            center = state.center - self.learning_rate * grad
        else:
            updates, state = use_state(self.optimizer.update)(state, grad, state.center)
            center = state.center + updates
        return state.update(center=center)
