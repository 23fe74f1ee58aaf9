"""LES — learned evolution strategy (Lange et al. 2023; reference ``es_variants/les.py:192-286``).

Recombination weights come from a small self-attention network over fitness
features (improvement flag, centred ranks, z-scores); per-dimension learning rates
for mean and σ come from an MLP over three evolution paths and a tanh time
embedding.  The reference loads meta-trained weights from a pickle that is absent
from its repository (``les.py:231-235``) — and pickles are never loaded here.  Pass
``net_params`` (nested dict of tensors, e.g. from safetensors) or
``net_ckpt_path`` (a ``.safetensors`` file with keys like
``recomb_weights.Dense_0.kernel``); without either, the networks are randomly
initialised from ``init_seed`` (a working but un-meta-trained LES).
"""
from __future__ import annotations

import math
import warnings

import torch

from ....core import Algorithm, State
from ....ops import random as rnd

TIMESCALES = (1, 3, 10, 30, 50, 100, 250, 500, 750, 1000, 1250, 1500, 2000)


def tanh_timestamp(x, t=None):
    t = torch.tensor(TIMESCALES, dtype=torch.float32, device=x.device) if t is None else t
    return torch.tanh(x.to(torch.float32) / t - 1.0)


def centered_rank_trafo(f):
    n = f.shape[0]
    r = torch.empty(n, device=f.device)
    r[torch.argsort(f, stable=True)] = torch.arange(n, dtype=torch.float32, device=f.device)
    return r / (n - 1) - 0.5


def z_score_trafo(a):
    return (a - torch.nanmean(a)) / (torch.sqrt(torch.nanmean((a - torch.nanmean(a)) ** 2)) + 1e-10)


def _dense(p, x):
    return x @ p["kernel"] + p["bias"]


def _init_dense(g, fan_in, fan_out):
    lim = math.sqrt(1.0 / fan_in)  # lecun-normal-like scale
    return {"kernel": torch.randn(fan_in, fan_out, generator=g) * lim, "bias": torch.zeros(fan_out)}


def init_les_params(seed=0, att_hidden=8, mlp_hidden=8, n_paths=3, n_feat=3):
    g = torch.Generator().manual_seed(seed)
    return {
        "recomb_weights": {"Dense_0": _init_dense(g, n_feat, att_hidden), "Dense_1": _init_dense(g, n_feat, att_hidden),
                           "Dense_2": _init_dense(g, n_feat, 1)},
        "lrate_modulation": {"Dense_0": _init_dense(g, 2 * n_paths + len(TIMESCALES), mlp_hidden),
                             "Dense_1": _init_dense(g, mlp_hidden, 1), "Dense_2": _init_dense(g, mlp_hidden, 1)},
    }


def _from_flat(flat):
    out = {}
    for k, v in flat.items():
        d = out
        parts = k.split(".")
        for p in parts[:-1]:
            d = d.setdefault(p, {})
        d[parts[-1]] = v
    return out


class LES(Algorithm):
    def __init__(self, pop_size, center_init, sigma_init=0.1, mean_decay=0.0, net_params=None, net_ckpt_path=None, init_seed=0):
        super().__init__()
        self.num_dims = center_init.shape[0]
        self.center_init = center_init
        self.popsize = pop_size
        self.sigma_init = sigma_init
        self.timescales = (0.1, 0.5, 0.9)
        if net_ckpt_path is not None:
            from safetensors.torch import load_file

            net_params = _from_flat(load_file(net_ckpt_path))
        if net_params is None:
            warnings.warn("LES: no meta-trained parameters given (the reference's pickle is not shipped); using random init")
            net_params = init_les_params(init_seed)
        dev = center_init.device
        conv = lambda t: {k: conv(v) if isinstance(v, dict) else torch.as_tensor(v, dtype=torch.float32, device=dev) for k, v in t.items()}
        self.params = conv(net_params)
        self._ts = torch.tensor(TIMESCALES, dtype=torch.float32, device=dev)
        self._path_lr = torch.tensor(self.timescales, dtype=torch.float32, device=dev)[None, :]

    def setup(self, key):
        dev = self.center_init.device
        paths = torch.zeros((self.num_dims, len(self.timescales)), device=dev)
        return State(key=key, sigma=self.sigma_init * torch.ones(self.num_dims, device=dev), mean=self.center_init.clone(),
                     path_c=paths, path_sigma=paths.clone(), best_fitness=torch.tensor(torch.finfo(torch.float32).max, device=dev),
                     best_member=self.center_init.clone(), gen_counter=torch.zeros((), dtype=torch.int64, device=dev),
                     x=torch.zeros((self.popsize, self.num_dims), device=dev), noises=torch.zeros((self.popsize, self.num_dims), device=dev))

    def ask(self, state):
        key, _ = rnd.split(state.key)
        noise = rnd.normal(state.key, (self.popsize, self.num_dims)).to(state.mean.device)
        x = state.mean + noise * state.sigma[None, :]
        return x, state.update(key=key, x=x, noises=noise)

    def _weights(self, feats):
        p = self.params["recomb_weights"]
        keys, queries, values = _dense(p["Dense_0"], feats), _dense(p["Dense_1"], feats), _dense(p["Dense_2"], feats)
        A = torch.softmax(queries @ keys.T / math.sqrt(feats.shape[0]), -1)
        return torch.softmax((A @ values).squeeze(-1), 0)[:, None]

    def _lrates(self, path_c, path_sigma, time_embed):
        p = self.params["lrate_modulation"]
        X = torch.cat([path_c, path_sigma, time_embed[None, :].expand(path_c.shape[0], -1)], 1)
        h = torch.relu(_dense(p["Dense_0"], X))
        return torch.sigmoid(_dense(p["Dense_1"], h)).squeeze(-1), torch.sigmoid(_dense(p["Dense_2"], h)).squeeze(-1)

    def _path_update(self, paths, diff):
        lr = self._path_lr
        return (1 - lr) * paths + (1 - lr) * diff[:, None]

    def tell(self, state, fitness):
        x = state.x
        feats = torch.stack([(fitness < state.best_fitness).to(torch.float32), centered_rank_trafo(fitness), z_score_trafo(fitness)], 1)
        w = self._weights(feats)
        path_c = self._path_update(state.path_c, (w * (x - state.mean)).sum(0))
        path_sigma = self._path_update(state.path_sigma, (w * (x - state.mean) / state.sigma).sum(0))
        lr_mean, lr_sigma = self._lrates(path_c, path_sigma, tanh_timestamp(state.gen_counter, self._ts))
        weighted_mean = (w * x).sum(0)
        weighted_sigma = torch.sqrt((w * (x - state.mean) ** 2).sum(0) + 1e-10)
        mean = state.mean + lr_mean * (weighted_mean - state.mean)
        sigma = torch.clamp(state.sigma + lr_sigma * (weighted_sigma - state.sigma), min=0)
        return state.update(mean=mean, sigma=sigma, path_c=path_c, path_sigma=path_sigma)
