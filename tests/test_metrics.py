"""Port of the reference's tests/test_metrics.py (same fronts, values and tolerances)
plus exact-HV cross-checks of the Monte-Carlo estimators."""
from math import isclose

import torch

from evoxmi import random as rnd
from evoxmi.metrics import GD, HV, IGD, GDPlus, IGDPlus, exact_hv


def test_gd_and_igd():
    pf = torch.tensor([[0, 5], [1, 4], [2, 3], [3, 2], [4, 1], [5.5, 0]])
    objs = torch.tensor([[0, 6], [5, 8], [4.3, 2]])
    assert isclose(GD(pf)(objs), 2.5669618, rel_tol=1e-4)
    assert isclose(GDPlus(pf)(objs), 2.5669618, rel_tol=1e-4)
    assert isclose(IGD(pf)(objs), 1.7367444, rel_tol=1e-4)
    assert isclose(IGDPlus(pf)(objs), 1.6073387, rel_tol=1e-4)
    assert isclose(GD(pf)(objs), IGD(objs)(pf), abs_tol=1e-4)


def test_hv():
    key = rnd.PRNGKey(0)
    ref = torch.tensor([-1.0, -1])
    objs = torch.tensor([[1.0, 9], [2, 2], [3, 1]])
    assert isclose(HV(ref, 100_000, "bounding_cube")(key, objs), 25, rel_tol=1e-2)
    assert isclose(HV(ref, 100_000, "each_cube")(key, objs), 25, rel_tol=1e-2)
    assert isclose(exact_hv(objs, ref), 25, rel_tol=1e-9)
    ref = torch.tensor([10, 9, 8.0])
    objs = torch.tensor([[0.1, 7, 0.3], [5.5, 0, 2.3], [-0.1, 1, -1], [3, 2, 5.5]])
    assert isclose(HV(ref, 100_000, "bounding_cube")(key, objs), 753, rel_tol=1e-2)
    assert isclose(HV(ref, 100_000, "each_cube")(key, objs), 753, rel_tol=1e-2)
    assert abs(exact_hv(objs, ref) - 753) < 2


def test_exact_hv_matches_mc_4d():
    g = torch.Generator().manual_seed(0)
    objs = torch.rand(12, 4, generator=g)
    ref = torch.ones(4) * 1.1
    ex = exact_hv(objs, ref)
    mc = float(HV(ref, 400_000, "bounding_cube")(rnd.PRNGKey(1), objs))
    assert abs(mc - ex) / ex < 0.02
