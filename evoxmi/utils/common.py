"""General utilities (reference ``src/evox/utils/common.py``).

Distance kernels use the GEMM form (``‖x‖² + ‖y‖² − 2xyᵀ``) so that on a GPU they
run on the matrix cores; ``dominate_relation`` is the tiled compare used by the
non-dominated sort (K9 of SURVEY §2.10).
"""
from __future__ import annotations

from collections.abc import Iterable
from typing import List, Union

import numpy as np
import torch

from ..core.algorithm import algorithm_has_init_ask  # noqa: F401  (re-export, common.py:15-19)
from ..core.module import Stateful
from ..core.state import State, tree_flatten, tree_leaves, tree_unflatten


def min_by(values, keys):
    """Row of ``values`` with the smallest ``keys`` (``common.py:22-31``)."""
    if isinstance(values, (list, tuple)):
        values = torch.cat(list(values))
        keys = torch.cat(list(keys))
    i = torch.argmin(keys)
    return values[i], keys[i]


def euclidean_dist(x, y):
    return torch.linalg.norm(x - y, dim=0)


def manhattan_dist(x, y):
    return torch.sum(torch.abs(x - y))


def chebyshev_dist(x, y):
    return torch.max(torch.abs(x - y))


def pairwise_euclidean_dist(x, y):
    """(N, M) Euclidean distances; GEMM form with a clamp for round-off."""
    xx = (x * x).sum(-1, keepdim=True)
    yy = (y * y).sum(-1, keepdim=True).T
    d2 = (xx + yy - 2.0 * (x @ y.T)).clamp_min_(0.0)
    return torch.sqrt(d2)


def pairwise_manhattan_dist(x, y):
    return torch.cdist(x, y, p=1)


def pairwise_chebyshev_dist(x, y):
    return torch.cdist(x, y, p=float("inf"))


def pair_max(a, b):
    return torch.max(a - b, dim=0).values


def cos_dist(x, y):
    """Cosine *similarity* matrix, as the reference computes it (``common.py:72-77``)."""
    xn = x / torch.linalg.norm(x, dim=-1, keepdim=True)
    yn = y / torch.linalg.norm(y, dim=-1, keepdim=True)
    return xn @ yn.T


def cal_max(x, y):
    """``out[i, j] = max_k (x[i, k] − y[j, k])`` (``common.py:80-82``)."""
    return (x[:, None, :] - y[None, :, :]).amax(-1)


def dominate(x, y):
    return bool(torch.all(x <= y) & torch.any(x < y))


def dominate_relation(x, y):
    """``A[i, j]`` is True iff ``x_i`` Pareto-dominates ``y_j`` (minimisation)."""
    le = (x[:, None, :] <= y[None, :, :]).all(-1)
    lt = (x[:, None, :] < y[None, :, :]).any(-1)
    return le & lt


def new_dist_mat(xs):
    return pairwise_euclidean_dist(xs, xs)


def compose(*functions):
    if len(functions) == 1 and isinstance(functions[0], Iterable):
        functions = functions[0]
    functions = list(functions)

    def composed(carry):
        for f in functions:
            carry = f(carry)
        return carry

    return composed


def rank(array: torch.Tensor) -> torch.Tensor:
    """Rank of each element of a 1-D tensor (0 = smallest)."""
    order = torch.argsort(array, stable=True)
    r = torch.empty_like(order)
    r[order] = torch.arange(order.shape[0], device=array.device)
    return r


def rank_based_fitness(raw_fitness: torch.Tensor) -> torch.Tensor:
    """Centred ranks in [−0.5, 0.5] (``common.py:143-147``)."""
    n = raw_fitness.shape[0]
    return rank(raw_fitness).to(torch.float32) / (n - 1) - 0.5


def _prod(xs):
    p = 1
    for x in xs:
        p *= x
    return p


class TreeAndVector:
    """Flat vector <-> parameter tree (``common.py:163-226``).

    Used as a ``sol_transform`` for neuroevolution: the algorithm works on flat
    ``(N, P)`` genomes, the problem receives a dict of ``(N, *shape)`` tensors.
    """

    def __init__(self, dummy_input):
        leaves, self.treedef = tree_flatten(dummy_input)
        self.shapes = [tuple(x.shape) for x in leaves]
        self.start_indices, self.slice_sizes = [], []
        index = 0
        for shape in self.shapes:
            self.start_indices.append(index)
            size = _prod(shape)
            self.slice_sizes.append(size)
            index += size
        self.total = index

    def to_vector(self, x):
        return torch.cat([t.reshape(-1) for t in tree_leaves(x)], dim=0)

    def batched_to_vector(self, x):
        return torch.cat([t.reshape(t.shape[0], -1) for t in tree_leaves(x)], dim=1)

    def to_tree(self, x):
        leaves = [x[s : s + n].reshape(shape) for s, n, shape in zip(self.start_indices, self.slice_sizes, self.shapes)]
        return tree_unflatten(leaves, self.treedef)

    def batched_to_tree(self, x):
        b = x.shape[0]
        leaves = [x[:, s : s + n].reshape(b, *shape) for s, n, shape in zip(self.start_indices, self.slice_sizes, self.shapes)]
        return tree_unflatten(leaves, self.treedef)


def parse_opt_direction(opt_direction: Union[str, List[str]]):
    """``"min"→1``, ``"max"→−1``; a list gives a per-objective tensor (``common.py:229-252``)."""
    if isinstance(opt_direction, str):
        if opt_direction == "min":
            return 1
        if opt_direction == "max":
            return -1
        raise ValueError(f"opt_direction is either 'min' or 'max', got {opt_direction}")
    if isinstance(opt_direction, (list, tuple)):
        out = []
        for d in opt_direction:
            if d == "min":
                out.append(1)
            elif d == "max":
                out.append(-1)
            else:
                raise ValueError(f"opt_direction is either 'min' or 'max', got {d}")
        return torch.tensor(out, dtype=torch.float32)
    raise ValueError(f"opt_direction should have type 'str' or 'list', got {type(opt_direction)}")


def frames2gif(frames, save_path, duration=0.1):
    """Write RGB frames to a GIF via Pillow (imageio is not a dependency here)."""
    from PIL import Image

    imgs = [Image.fromarray(np.asarray(f, dtype=np.uint8)) for f in frames]
    imgs[0].save(save_path, save_all=True, append_images=imgs[1:], duration=int(duration * 1000), loop=0)
    return save_path


class AggregationFunction:
    """Decomposition scalarisers (``common.py:271-317``): PBI (θ=5), Tchebycheff,
    normalised Tchebycheff, modified Tchebycheff, weighted sum."""

    def __init__(self, function_name: str):
        table = {
            "pbi": self.pbi,
            "tchebycheff": self.tchebycheff,
            "tchebycheff_norm": self.tchebycheff_norm,
            "modified_tchebycheff": self.modified_tchebycheff,
            "weighted_sum": self.weighted_sum,
        }
        if function_name not in table:
            raise ValueError("Unsupported function")
        self.name = function_name
        self.function = table[function_name]

    @staticmethod
    def pbi(f, w, z, *args):
        norm_w = torch.linalg.norm(w, dim=-1)
        f = f - z
        d1 = (f * w).sum(-1) / norm_w
        d2 = torch.linalg.norm(f - d1[..., None] * w / norm_w[..., None], dim=-1)
        return d1 + 5 * d2

    @staticmethod
    def tchebycheff(f, w, z, *args):
        return (torch.abs(f - z) * w).amax(-1)

    @staticmethod
    def tchebycheff_norm(f, w, z, z_max, *args):
        return (torch.abs(f - z) / (z_max - z) * w).amax(-1)

    @staticmethod
    def modified_tchebycheff(f, w, z, *args):
        return (torch.abs(f - z) / w).amax(-1)

    @staticmethod
    def weighted_sum(f, w, *args):
        return (f * w).sum(-1)

    def __call__(self, *args, **kwargs):
        return self.function(*args, **kwargs)


def to_x32_if_needed(values):
    """Down-cast float64/int64 arrays from host callbacks (``utils/io.py:6-26``)."""
    if isinstance(values, torch.Tensor):
        if values.dtype == torch.float64:
            return values.float()
        return values
    if isinstance(values, np.ndarray):
        if values.dtype == np.float64:
            return values.astype(np.float32)
        if values.dtype == np.int64:
            return values.astype(np.int32)
    return values


def x32_func_call(func):
    def inner(*args, **kwargs):
        return to_x32_if_needed(func(*args, **kwargs))

    return inner
