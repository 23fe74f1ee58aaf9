"""Port of the reference's tests/test_gaussian_process.py (same data, optimiser and
golden values) plus a classification sanity check (parity unpinned)."""
import torch

from evoxmi.operators.gaussian_process import Gaussian, GPClassification, GPRegression
from evoxmi.utils import optim


def test_gp():
    x = torch.arange(5.0)[:, None]
    pre_x = torch.tensor([4.0, 5, 6])[:, None]
    y = (torch.arange(5.0) * 6)[:, None]
    model = GPRegression(likelihood=Gaussian(num_datapoints=len(x)))
    model.fit(x, y, optimzer=optim.sgd(0.001, nesterov=True))
    _, mean, std = model.predict(pre_x)
    assert abs(float(mean[1]) - 2.90525) < 0.001
    assert abs(float(std[1]) - 4.80366) < 0.001


def test_gp_classification_separable():
    x = torch.linspace(-3, 3, 40)[:, None]
    y = (x[:, 0] > 0).to(torch.float32)
    model = GPClassification().fit(x, y)
    _, p, _ = model.predict(torch.tensor([[-2.0], [2.0]]))
    assert float(p[0]) < 0.3 and float(p[1]) > 0.7
