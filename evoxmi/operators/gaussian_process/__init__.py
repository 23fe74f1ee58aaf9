"""Exact Gaussian-process regression and (MAP, probit) GP classification in PyTorch
(reference ``operators/gaussian_process/`` wraps gpjax, which is not available here).

Kernels, likelihoods and the optimisation protocol follow gpjax's defaults so that
the reference's golden regression test reproduces: RBF(lengthscale = 1, variance = 1),
Gaussian(obs_stddev = 1), zero mean, parameters optimised in softplus-unconstrained
space by the given first-order optimiser (250 iterations for regression, 500 for
classification) on the negative (conjugate) marginal log-likelihood.
"""
from .kernels import RBF, Linear, Matern52
from .likelihoods import Bernoulli, Gaussian
from .regression import GPRegression
from .classification import GPClassification

__all__ = ["RBF", "Linear", "Matern52", "Gaussian", "Bernoulli", "GPRegression", "GPClassification"]
