"""Hierarchical, immutable module state.

Behavioural parity with the reference ``State`` (``src/evox/core/state.py:17-234``):
a node holds its own fields (a dict or a dataclass), a mapping of named child
states and the ``state_id`` of the module that owns it.  Updates are functional
(``update`` / ``replace`` / ``update_child`` return new nodes), ``find_path_to`` /
``update_path`` locate a sub-state by node id, and mutation raises ``TypeError``.

MI355X-first differences:

* leaves are ``torch.Tensor`` (usually resident in HBM) or plain Python scalars;
  the tree is registered with ``torch.utils._pytree`` so the generic tree
  utilities (``tree_map``, flattening for hipGraph static buffers,
  checkpointing) see every tensor;
* ``save`` / ``load`` use the version-tagged manifest + safetensors format of
  :mod:`evoxmi.core.checkpoint` instead of pickle, so a checkpoint never
  executes code when it is read.
"""
from __future__ import annotations

import dataclasses
from copy import copy
from pprint import pformat
from typing import Any, Optional, Tuple, Union

import torch
import torch.utils._pytree as pytree


def is_magic_method(name: str) -> bool:
    return name.startswith("__") and name.endswith("__")


class State:
    """Immutable hierarchical state.

    ``State(x=1, y=2)`` builds a node from keyword arguments, ``State(dc)`` from a
    dataclass instance.  Use ``update`` (or ``replace``) to derive a new state.
    """

    EMPTY: dict = {}

    def __init__(self, _dataclass=None, /, **kwargs) -> None:
        if _dataclass is not None:
            assert dataclasses.is_dataclass(_dataclass), "positional argument must be a dataclass"
            self.__dict__["_state_dict"] = _dataclass
        else:
            self.__dict__["_state_dict"] = kwargs
        self.__dict__["_child_states"] = State.EMPTY
        self.__dict__["_state_id"] = None

    # --- unsafe in-place constructors (used while building the tree) -------------
    def _set_state_dict_mut(self, state_dict) -> "State":
        self.__dict__["_state_dict"] = state_dict
        return self

    def _set_child_states_mut(self, child_states: dict) -> "State":
        self.__dict__["_child_states"] = child_states
        return self

    def _set_state_id_mut(self, state_id) -> "State":
        self.__dict__["_state_id"] = state_id
        return self

    # --- functional updates ---------------------------------------------------------
    def update(self, **kwargs) -> "State":
        if dataclasses.is_dataclass(self._state_dict):
            return copy(self)._set_state_dict_mut(dataclasses.replace(self._state_dict, **kwargs))
        return copy(self)._set_state_dict_mut({**self._state_dict, **kwargs})

    def replace(self, **kwargs) -> "State":
        return self.update(**kwargs)

    def has_child(self, name: str) -> bool:
        return name in self._child_states

    def get_child_state(self, name: str) -> "State":
        return self._child_states[name]

    def update_child(self, name: str, child_state: "State") -> "State":
        return copy(self)._set_child_states_mut({**self._child_states, name: child_state})

    def keys(self):
        if dataclasses.is_dataclass(self._state_dict):
            return [f.name for f in dataclasses.fields(self._state_dict)]
        return list(self._state_dict.keys())

    # --- path search ----------------------------------------------------------------
    def find_path_to(self, node_id: int, hint: Optional[str] = None):
        """Return ``(path, state)`` of the node whose ``state_id == node_id``."""
        if node_id == self._state_id:
            return node_id, self
        if hint in self._child_states and node_id == self._child_states[hint]._state_id:
            return (hint, node_id), self._child_states[hint]
        for child_id, child_state in self._child_states.items():
            result = child_state.find_path_to(node_id)
            if result is not None:
                path, state = result
                return (child_id, path), state
        return None

    def update_path(self, path, new_state: "State") -> "State":
        if isinstance(path, int):
            assert path == self._state_id
            return new_state
        if isinstance(path, tuple):
            child_id, sub = path
            return self.update_child(child_id, self._child_states[child_id].update_path(sub, new_state))
        raise ValueError("path must be a tuple or an int")

    # --- attribute access -----------------------------------------------------------
    def __getattr__(self, key: str) -> Any:
        if is_magic_method(key):
            return super().__getattribute__(key)
        sd = self.__dict__["_state_dict"]
        if dataclasses.is_dataclass(sd):
            return getattr(sd, key)
        try:
            return sd[key]
        except KeyError:
            raise AttributeError(key) from None

    def __getitem__(self, key: str) -> Any:
        return getattr(self, key)

    def __contains__(self, key: str) -> bool:
        return key in self.keys()

    def index(self, index) -> "State":
        """Apply ``x[index]`` to every tensor leaf."""
        return tree_map(lambda x: x[index] if isinstance(x, torch.Tensor) else x, self)

    def slice(self, begin: int, end: int) -> "State":
        if isinstance(begin, int) and isinstance(end, int):
            return tree_map(lambda x: x[begin:end] if isinstance(x, torch.Tensor) else x, self)
        raise TypeError(f"begin and end must be int, got {type(begin)} and {type(end)}")

    def __setattr__(self, _k, _v):
        raise TypeError("State is immutable")

    def __setitem__(self, _k, _v):
        raise TypeError("State is immutable")

    # --- printing -------------------------------------------------------------------
    def __repr__(self) -> str:
        if self is State.EMPTY:
            return "State.empty"
        kids = ",".join(f"{k!r}: {v!r}" for k, v in self._child_states.items())
        return f"State({self._state_dict!r}, {{{kids}}})"

    def __str__(self) -> str:
        return f"State{pformat(self.sprint_tree())}"

    def sprint_tree(self):
        if self is State.EMPTY:
            return "State.empty"
        return self._state_dict, {k: v.sprint_tree() for k, v in self._child_states.items()}

    def __eq__(self, other) -> bool:
        if not isinstance(other, State):
            return False
        a, b = tree_leaves(self), tree_leaves(other)
        if len(a) != len(b) or tree_structure(self) != tree_structure(other):
            return False
        for x, y in zip(a, b):
            if isinstance(x, torch.Tensor) or isinstance(y, torch.Tensor):
                if not (isinstance(x, torch.Tensor) and isinstance(y, torch.Tensor)):
                    return False
                if x.shape != y.shape or not torch.equal(x.cpu(), y.cpu()):
                    return False
            elif x != y:
                return False
        return True

    __hash__ = None

    # --- persistence (see evoxmi.core.checkpoint) -----------------------------------
    def save(self, path: str) -> None:
        from .checkpoint import save_state

        save_state(self, path)

    def load(self, path: str, map_location=None) -> "State":
        from .checkpoint import load_state

        return load_state(path, map_location=map_location)

    # --- device helpers ---------------------------------------------------------------
    def to(self, device) -> "State":
        return tree_map(lambda x: x.to(device) if isinstance(x, torch.Tensor) else x, self)


# ----------------------------------------------------------------------------------------
# pytree registration
# ----------------------------------------------------------------------------------------
def _state_flatten(s: State):
    return [s._state_dict, s._child_states], s._state_id


def _state_unflatten(children, state_id):
    state_dict, child_states = children
    return State()._set_state_id_mut(state_id)._set_state_dict_mut(state_dict)._set_child_states_mut(child_states)


def _state_flatten_with_keys(s: State):
    return [(pytree.GetAttrKey("_state_dict"), s._state_dict), (pytree.GetAttrKey("_child_states"), s._child_states)], s._state_id


pytree.register_pytree_node(
    State,
    _state_flatten,
    _state_unflatten,
    serialized_type_name="evoxmi.State",
    flatten_with_keys_fn=_state_flatten_with_keys,
)


def tree_map(fn, tree, *rest):
    return pytree.tree_map(fn, tree, *rest)


def tree_leaves(tree):
    return pytree.tree_leaves(tree)


def tree_flatten(tree):
    return pytree.tree_flatten(tree)


def tree_unflatten(leaves, spec):
    return pytree.tree_unflatten(leaves, spec)


def tree_structure(tree):
    return pytree.tree_structure(tree)
