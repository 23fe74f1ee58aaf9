"""Golden values of the reference's tests/test_maf.py (key = PRNGKey(1),
data = uniform(key, (3, 12)), m = 3), with the same input data regenerated bit-exactly
by tests/jax_threefry.py.  The reference's PF checks of MaF1/2/3 are one-sided
(``r2[1,1] - v < 1e-4``); here every PF value is checked two-sided."""
import pytest
import torch

from jax_threefry import PRNGKey, uniform
from evoxmi.problems.numerical import maf as M

DATA = torch.tensor(uniform(PRNGKey(1), (3, 12)))
n, d = DATA.shape
m = 3

GOLD = [
    ("MaF1", 1.8404, 0.9867, "abs"), ("MaF2", 0.6237, 0.3458, "abs"), ("MaF3", 2.1354973e11, 1.8255e-04, "rel"),
    ("MaF4", 1.9944e03, 3.9460, "abs2"), ("MaF5", 2.1819e-40, 0.0540, "abs"), ("MaF6", 55.8732, 2.3586e-04, "abs"),
    ("MaF7", 0.3915, 0.0, "abs"), ("MaF8", 1.2490, 0.0545, "abs"), ("MaF9", 0.3118, 0.0351, "rel"),
    ("MaF10", 1.0060, 0.0483, "abs"), ("MaF11", 0.6342, 0.1021, "abs"), ("MaF12", 3.4703, 0.0540, "abs"),
    ("MaF13", 0.8246, 0.0135, "abs"), ("MaF14", 0.1718, 0.0133, "abs"), ("MaF15", 0.8123, 0.9865, "abs"),
]


def test_inside():
    assert not M.inside(8.5, 1.0, 0.0)
    assert not M.inside(8.5, 0.0, 1.0)
    assert M.inside(0.5, 0.0, 1.0)
    assert M.inside(0.5, 1.0, 0.0)
    assert not M.inside(1.0, 1.0, 0.0)
    assert M.inside(0.0, 1.0, 0.0)
    assert not M.inside(1.0, 0.0, 1.0)
    assert M.inside(0.0, 0.0, 1.0)


def test_ray_intersect_segment():
    p = torch.tensor([0.0, 0.0])
    t = lambda a, b: bool(M.ray_intersect_segment(p, torch.tensor(a), torch.tensor(b)))
    assert not t([1.0, 1.0], [1.0, 2.0])
    assert t([1.0, 1.0], [-1.0, -1.0])
    assert t([1.0, 1.0], [1.0, -1.0])
    assert not t([1.0, 0.0], [1.0, -1.0])
    assert t([1.0, 0.0], [1.0, 1.0])
    assert t([1.0, 1.0], [1.0, 0.0])


def test_point_in_polygon():
    poly = torch.tensor([[0, 1.0], [-0.5, -1], [0.5, -1]])
    assert M.point_in_polygon(poly, torch.tensor([0.0, 0.0]))
    assert not M.point_in_polygon(poly, torch.tensor([1.0, -1.0]))
    assert M.point_in_polygon(poly, torch.tensor([0.0, 1.0]))
    assert not M.point_in_polygon(poly, torch.tensor([-1.0, 1.0]))


@pytest.mark.parametrize("name,v_eval,v_pf,mode", GOLD)
def test_maf_golden(name, v_eval, v_pf, mode):
    prob = getattr(M, name)(d=d, m=m)
    r1, _ = prob.evaluate(None, DATA)
    r2 = prob.pf()
    assert r1.shape == (3, 3)
    assert r2.shape[1] == 3
    got = float(r1[1, 1])
    if mode == "rel":
        assert abs(got - v_eval) / abs(v_eval) < 1e-4
    elif mode == "abs2":
        assert abs(got - v_eval) < 1e-2
    else:
        assert abs(got - v_eval) < 1e-4
    assert abs(float(r2[1, 1]) - v_pf) < 1e-4
