"""Supervised-learning neuroevolution problem (reference ``supervised_learning/tfds.py:28-135``).

The population's loss on the next mini-batch of a dataset.  TFDS / grain are not in
this stack, so the data source is any of:

* a mapping of equal-length tensors/arrays (e.g. ``{"image": X, "label": y}``),
* a ``torch.utils.data.Dataset`` returning such mappings,
* a locally available Hugging Face ``datasets`` dataset (``dataset="<name or path>"``),
  loaded with ``datasets.load_dataset`` (no network access is attempted beyond what
  the local cache provides).

Batches are drawn by a seeded shuffled sampler with ``drop_remainder`` semantics and
moved to the population's device; ``loss_func(params, batch)`` is applied to the
whole population at once when ``batched_loss=True`` (else per individual, the
reference's ``vmap``).
"""
from __future__ import annotations

from typing import Any, Callable, List, Optional

import numpy as np
import torch

from ....core import Problem, State


class _Sampler:
    def __init__(self, n, batch_size, seed):
        self.n, self.bs = n, batch_size
        self.rng = np.random.default_rng(seed)
        self.perm, self.pos = self.rng.permutation(n), 0

    def next(self):
        if self.pos + self.bs > self.n:
            self.perm, self.pos = self.rng.permutation(self.n), 0
        idx = self.perm[self.pos : self.pos + self.bs]
        self.pos += self.bs
        return idx


class TensorflowDataset(Problem):
    def __init__(self, dataset: Any, batch_size: int, loss_func: Callable, split: str = "train", operations: List[Any] = (),
                 datadir: Optional[str] = None, seed: int = 0, try_gcs: bool = False, batched_loss: bool = False):
        super().__init__()
        self.batch_size, self.loss_func, self.operations, self.batched_loss = batch_size, loss_func, list(operations), batched_loss
        if isinstance(dataset, str):
            try:
                import datasets as hf
            except ImportError as e:  # pragma: no cover
                raise ImportError("loading a dataset by name needs the `datasets` package and a local copy") from e
            ds = hf.load_dataset(dataset, split=split, cache_dir=datadir)
            dataset = {k: np.asarray(ds[k]) for k in ds.column_names}
        if isinstance(dataset, dict):
            self.data = {k: torch.as_tensor(np.asarray(v)) for k, v in dataset.items()}
            n = len(next(iter(self.data.values())))
            self._get = lambda idx: {k: v[torch.as_tensor(idx)] for k, v in self.data.items()}
        else:
            n = len(dataset)
            self._get = lambda idx: torch.utils.data.default_collate([dataset[int(i)] for i in idx])
        self.sampler = _Sampler(n, batch_size, seed)

    def setup(self, key):
        return State(key=key)

    def _next_data(self):
        batch = self._get(self.sampler.next())
        for op in self.operations:
            batch = op(batch)
        return batch

    def evaluate(self, state, pop):
        leaves = [x for x in torch.utils._pytree.tree_leaves(pop) if isinstance(x, torch.Tensor)]
        dev = leaves[0].device
        batch = torch.utils._pytree.tree_map(lambda x: x.to(dev) if isinstance(x, torch.Tensor) else x, self._next_data())
        if self.batched_loss:
            return self.loss_func(pop, batch), state
        n = leaves[0].shape[0]
        loss = torch.stack([torch.as_tensor(self.loss_func(torch.utils._pytree.tree_map(lambda x: x[i], pop), batch)) for i in range(n)])
        return loss.to(dev), state
