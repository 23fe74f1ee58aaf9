"""Stateful modules and state scoping.

Parity map (reference ``src/evox/core/module.py``):

* :func:`use_state` — ``module.py:15-87``: locate the callee's sub-state by node id
  (with a name hint), run the method on it, merge the returned sub-state back.
  ``index=`` addresses one member of a stacked (batched) module.
* :func:`jit_method` / :func:`jit_class` — ``module.py:90-137``.  There is no
  tracing compiler here: a generation is made launch-cheap by hipGraph capture
  (:class:`evoxmi.workflows.StdWorkflow` ``graph=True``), so these decorators only
  tag the class as "side-effect free between state in and state out".
* :func:`dataclass`, ``Static``, ``Stack`` — ``module.py:140-209``.
* :class:`Stateful` — ``module.py:212-358``: deterministic recursive ``init`` over
  sub-modules in **sorted attribute-name order** (so node ids, hence checkpoint
  paths, are stable), one PRNG-key split per sub-module, ``setup(key)`` per node.
"""
from __future__ import annotations

import dataclasses
from collections import namedtuple
from functools import partial, wraps
from typing import Annotated, Any, Callable, TypeVar, get_type_hints

import torch
import torch.utils._pytree as pytree

from .state import State, tree_map


def _index_leaf(x, index):
    return x[index] if isinstance(x, torch.Tensor) else x


def _set_index_leaf(batch, new, index):
    if isinstance(batch, torch.Tensor):
        out = batch.clone()
        out[index] = new
        return out
    return new


def use_state(func: Callable, index: int = None):
    """Scope ``func`` to the sub-state of the module it belongs to.

    ``use_state(self.algorithm.ask)(state)`` finds ``state``'s node whose id equals
    ``self.algorithm``'s node id, calls ``ask`` on it, and grafts the returned
    sub-state back into the full tree.
    """

    err_msg = "Expect last return value must be State, got {}"

    def wrapper(self, state: State, *args, **kwargs):
        assert isinstance(state, State), f"The first argument must be `State`, got {type(state)}"
        if getattr(self, "_node_id", None) is None and not isinstance(self, (list, tuple)):
            raise ValueError(f"{self} is not initialized, did you forget to call `init`?")
        node_id = self._node_id if not isinstance(self, (list, tuple)) else self[0]._node_id
        module_name = self._module_name if not isinstance(self, (list, tuple)) else self[0]._module_name
        found = state.find_path_to(node_id, module_name)
        if found is None:
            raise ValueError(f"state for node {node_id} ({module_name}) not found")
        path, matched_state = found

        if index is not None:
            extracted_state = tree_map(partial(_index_leaf, index=index), matched_state)
        else:
            extracted_state = matched_state

        if hasattr(func, "__self__"):
            rv = func(extracted_state, *args, **kwargs)
        else:
            this_module = self[index] if (index is not None and isinstance(self, (list, tuple))) else self
            rv = func(this_module, extracted_state, *args, **kwargs)

        if not isinstance(rv, tuple):
            assert isinstance(rv, State), err_msg.format(type(rv))
            aux, new_state = None, rv
        else:
            assert isinstance(rv[-1], State), err_msg.format(type(rv[-1]))
            aux, new_state = rv[:-1], rv[-1]

        if index is not None:
            new_state = tree_map(partial(_set_index_leaf, index=index), matched_state, new_state)

        state = state.update_path(path, new_state)
        return state if aux is None else (*aux, state)

    if hasattr(func, "__self__"):
        return wraps(func)(partial(wrapper, func.__self__))
    return wraps(func)(wrapper)


def jit_method(method: Callable) -> Callable:
    """API-compatibility decorator (see module docstring): returns ``method`` tagged."""
    try:
        method._evoxmi_pure = True
    except AttributeError:
        pass
    return method


def jit_class(cls):
    """Tag every public method of ``cls`` as pure (state in → state out)."""
    cls._evoxmi_pure_class = True
    return cls


StaticAnnotation = "evoxmi_dataclass_static_field"
Static = Annotated[TypeVar("T"), StaticAnnotation]
StackAnnotation = "evoxmi_dataclass_stack_field"
Stack = Annotated[TypeVar("T"), StackAnnotation]


def _has_annotation(type_hint, annotation) -> bool:
    return hasattr(type_hint, "__metadata__") and annotation in type_hint.__metadata__


def dataclass(cls, *args, **kwargs):
    """A dataclass registered as a pytree; ``Static[...]`` fields go to the tree spec."""
    cls = dataclasses.dataclass(cls, *args, **kwargs)
    hints = get_type_hints(cls, include_extras=True)
    field_info = [(f.name, f.init, _has_annotation(hints[f.name], StaticAnnotation)) for f in dataclasses.fields(cls)]
    field_info.append(("_node_id", False, True))
    field_info.append(("_module_name", False, True))

    def flatten(obj):
        children, aux = [], []
        for name, _, is_static in field_info:
            value = getattr(obj, name, None)
            (aux if is_static else children).append(value)
        return children, tuple(aux)

    def unflatten(children, aux):
        it_aux, it_ch = iter(aux), iter(children)
        obj = object.__new__(cls)
        for name, _, is_static in field_info:
            object.__setattr__(obj, name, next(it_aux) if is_static else next(it_ch))
        return obj

    pytree.register_pytree_node(cls, flatten, unflatten, serialized_type_name=f"{cls.__module__}.{cls.__qualname__}")
    from .checkpoint import register_dataclass

    register_dataclass(cls)
    return cls


class Stateful:
    """Base class for every evoxmi module (algorithms, problems, workflows, ...).

    Hyper-parameters live on ``self`` (set in ``__init__``); mutable data lives in
    the :class:`State` returned by ``setup``.  ``init(key)`` builds the whole tree.
    """

    def __init__(self):
        super().__init__()
        object.__setattr__(self, "_node_id", None)
        object.__setattr__(self, "_module_name", None)

    def setup(self, key) -> State:
        return State()

    def _submodules(self):
        Sub = namedtuple("Sub", ["name", "module", "stacked"])
        subs = []
        if dataclasses.is_dataclass(self):
            hints = get_type_hints(type(self), include_extras=True)
            for f in dataclasses.fields(self):
                attr = getattr(self, f.name)
                stacked = _has_annotation(hints.get(f.name), StackAnnotation)
                if isinstance(attr, Stateful) or (stacked and isinstance(attr, (list, tuple))):
                    subs.append(Sub(f.name, attr, stacked))
        else:
            for name, attr in vars(self).items():
                if name.startswith("_"):
                    continue
                if isinstance(attr, Stateful):
                    subs.append(Sub(name, attr, False))
                elif isinstance(attr, StackedModules):
                    subs.append(Sub(name, attr, True))
        subs.sort(key=lambda s: s.name)
        return subs

    def _recursive_init(self, key, node_id: int, module_name, no_state: bool):
        from ..ops import random as _rand

        object.__setattr__(self, "_node_id", node_id)
        object.__setattr__(self, "_module_name", module_name)
        child_states = {}
        for name, attr, stacked in self._submodules():
            if key is None:
                subkey = None
            else:
                key, subkey = _rand.split(key)
            if stacked:
                members = list(attr)
                subkeys = _rand.split(subkey, len(members)) if subkey is not None else [None] * len(members)
                first_id = node_id + 1
                states = []
                last_id = node_id
                for m, k in zip(members, subkeys):
                    st, last_id = m._recursive_init(k, first_id, name, no_state)
                    states.append(st)
                node_id = last_id
                if not no_state:
                    child_states[name] = stack_states(states)
            else:
                st, node_id = attr._recursive_init(subkey, node_id + 1, name, no_state)
                if not no_state:
                    assert isinstance(st, State), "setup method must return a State"
                    child_states[name] = st
        if no_state:
            return None, node_id
        st = self.setup(key)
        assert isinstance(st, State), f"{type(self).__name__}.setup must return a State"
        return st._set_state_id_mut(self._node_id)._set_child_states_mut(child_states), node_id

    def init(self, key=None, no_state: bool = False) -> State:
        """Initialise this module and all sub-modules; returns the state tree."""
        state, _ = self._recursive_init(key, 0, None, no_state)
        return state

    @classmethod
    def stack(cls, stateful_objs, axis: int = 0):
        """Stack dataclass modules leaf-wise (reference ``module.py:341-349``)."""
        for obj in stateful_objs:
            assert dataclasses.is_dataclass(obj), "All objects must be dataclasses"
        return tree_map(lambda *xs: torch.stack(xs, dim=axis) if isinstance(xs[0], torch.Tensor) else xs[0], *stateful_objs)

    def __len__(self) -> int:
        assert dataclasses.is_dataclass(self), "Length is only supported for dataclass"
        leaves = [x for x in pytree.tree_leaves(self) if isinstance(x, torch.Tensor)]
        return len(leaves[0])


class StackedModules(list):
    """A batch of identically-structured sub-modules sharing one node id.

    Non-dataclass modules mark a ``Stack`` field by wrapping the list of members in
    ``StackedModules``; their states are stacked leaf-wise along a new leading dim
    and ``use_state(fn, index=i)`` addresses member ``i``.
    """


def stack_states(states):
    def _stack(*xs):
        if isinstance(xs[0], torch.Tensor):
            return torch.stack(xs, dim=0)
        return xs[0]

    return tree_map(_stack, *states)
