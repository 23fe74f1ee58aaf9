"""Port of the reference's tests/test_state.py semantics (hierarchical init, use_state
scoping, immutability, pytree round-trip) plus the safetensors checkpoint format."""
import os

import pytest
import torch

from evoxmi import Stateful, State, use_state, dataclass, Static
from evoxmi import random as rnd
from evoxmi.core.state import tree_flatten, tree_unflatten, tree_map


class Leaf(Stateful):
    def __init__(self, v):
        super().__init__()
        self.v = v

    def setup(self, key):
        return State(c=self.v, t=torch.arange(3) * self.v)

    def inc(self, state):
        return state.update(c=state.c + 1)

    def get(self, state):
        return state.c, state


class Mid(Stateful):
    def __init__(self):
        super().__init__()
        self.b_leaf = Leaf(2)
        self.a_leaf = Leaf(1)

    def setup(self, key):
        return State(m=0)


class Top(Stateful):
    def __init__(self):
        super().__init__()
        self.mid = Mid()
        self.leaf = Leaf(5)


def test_basic_tree_and_node_ids():
    top = Top()
    st = top.init(rnd.PRNGKey(0))
    # sorted attribute names: leaf < mid ; a_leaf < b_leaf
    assert top._node_id == 0
    assert top.leaf._node_id == 1
    assert top.mid._node_id == 2
    assert top.mid.a_leaf._node_id == 3
    assert top.mid.b_leaf._node_id == 4
    assert st.get_child_state("mid").get_child_state("b_leaf").c == 2
    assert set(st._child_states) == {"leaf", "mid"}
    assert set(st.get_child_state("mid")._child_states) == {"a_leaf", "b_leaf"}


def test_use_state_scoping():
    top = Top()
    st = top.init(rnd.PRNGKey(0))
    st2 = use_state(top.mid.b_leaf.inc)(st)
    assert st2.get_child_state("mid").get_child_state("b_leaf").c == 3
    assert st.get_child_state("mid").get_child_state("b_leaf").c == 2  # immutable
    c, st3 = use_state(top.leaf.get)(st2)
    assert c == 5


def test_immutable():
    s = State(x=1)
    with pytest.raises(TypeError):
        s.x = 2
    with pytest.raises(TypeError):
        s["x"] = 2
    assert s.update(x=3).x == 3 and s.x == 1


def test_repr_and_str():
    s = State(x=1)
    assert repr(s) == "State({'x': 1}, {})"
    assert "x" in str(s)


def test_pytree_roundtrip():
    st = Top().init(rnd.PRNGKey(1))
    leaves, spec = tree_flatten(st)
    st2 = tree_unflatten(leaves, spec)
    assert st2 == st
    st3 = tree_map(lambda x: x * 2 if isinstance(x, torch.Tensor) else x, st)
    assert torch.equal(st3.get_child_state("leaf").t, torch.tensor([0, 10, 20]))


@dataclass
class DState:
    a: torch.Tensor
    n: Static[int]


def test_dataclass_state_and_checkpoint(tmp_path):
    top = Top()
    st = top.init(rnd.PRNGKey(3))
    st = st.update(extra=State(DState(a=torch.ones(2), n=3)), scal=1.5, tup=(1, torch.zeros(2)))
    p = os.path.join(tmp_path, "ck.safetensors")
    st.save(p)
    back = State().load(p)
    assert back == st
    assert back._state_id == st._state_id
    assert back.get_child_state("mid")._state_id == st.get_child_state("mid")._state_id
    assert isinstance(back.extra._state_dict, DState)


def test_find_and_update_path():
    top = Top()
    st = top.init(rnd.PRNGKey(0))
    path, sub = st.find_path_to(top.mid.a_leaf._node_id, "a_leaf")
    assert sub.c == 1
    st2 = st.update_path(path, sub.update(c=10))
    assert st2.get_child_state("mid").get_child_state("a_leaf").c == 10


def test_checkpoint_dict_keys_do_not_collide(tmp_path):
    """A dict key containing '.' must not overwrite another leaf's tensor, and non-str
    dict keys come back with their type (advisor finding on checkpoint.py)."""
    import torch

    from evoxmi.core import State
    from evoxmi.core.checkpoint import load_state, save_state

    st = State(tab={"a.b": torch.ones(2), "a": {"b": torch.zeros(3)}, 7: torch.full((1,), 7.0)})
    p = str(tmp_path / "ck.safetensors")
    save_state(st, p)
    back = load_state(p)
    tab = back.tab
    assert torch.equal(tab["a.b"], torch.ones(2))
    assert torch.equal(tab["a"]["b"], torch.zeros(3))
    assert 7 in tab and torch.equal(tab[7], torch.full((1,), 7.0))
