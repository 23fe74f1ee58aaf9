"""Golden values of the reference's tests/test_lsmop.py, recomputed on the same input
data (regenerated bit-exactly with a numpy threefry: see tests/jax_threefry.py)."""
import numpy as np
import pytest
import torch

from jax_threefry import PRNGKey, uniform
from evoxmi.problems.numerical.lsmop import LSMOP1, LSMOP2, LSMOP3, LSMOP4, LSMOP5, LSMOP6, LSMOP7, LSMOP8, LSMOP9

upper = np.concatenate([np.ones(2), 10 * np.ones(298)]).astype(np.float32)
DATA = torch.tensor(uniform(PRNGKey(0), (100, 300), 0.0, upper))

GOLD = [
    (LSMOP1, 12.5981, 21.2454, False), (LSMOP2, 0.6876, 0.4688, False), (LSMOP3, 5.3782496e04, 26.0379, True),
    (LSMOP4, 0.5550, 0.8865, False), (LSMOP5, 2.6036, 10.7802, False), (LSMOP6, 1.7095365e03, 2.5482053e04, True),
    (LSMOP7, 1.4722900e04, 1.3406048, "a"), (LSMOP8, 1.9358, 0.8251, False), (LSMOP9, 0.0523, 217.5438, False),
]


@pytest.mark.parametrize("cls,v11,v12,rel", GOLD)
def test_lsmop_golden(cls, v11, v12, rel):
    prob = cls(d=300, m=3)
    r, _ = prob.evaluate(None, DATA)
    assert r.shape == (100, 3)
    if rel is True:
        assert abs(r[1, 1].item() - v11) / v11 < 1e-5
        assert abs(r[1, 2].item() - v12) / v12 < 1e-5
    elif rel == "a":
        assert abs(r[1, 1].item() - v11) / v11 < 1e-5
        assert abs(r[1, 2].item() - v12) < 1e-4
    else:
        assert abs(r[1, 1].item() - v11) < 1e-4
        assert abs(r[1, 2].item() - v12) < 1e-4
    pf = prob.pf()
    assert pf.shape[1] == 3


def test_lsmop_quirk_default_d():
    p = LSMOP1(m=3)
    assert p.d == 7 and p.sublen[0] > 0  # groups computed with d = 300, then d reset (reference lsmop.py:116-125)
