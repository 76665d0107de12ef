"""Distributions of the reference (drop-in for smcdet/distributions.py).

These are small elementwise utilities kept for API compatibility
(`DiscreteUniform` :5-19, `TruncatedDiagonalMVN` :22-58, `TruncatedPareto`
:61-89).  They run as torch elementwise ops on whatever device their tensors
live on.  Their formulas are the API (a user's code calls them), so they
follow the reference line for line; tests/test_dropin_distributions.py pins
them bit for bit to the reference's own outputs (tests/golden/distributions.npz).
The hot path does not call them: the MH kernel samples and scores
its truncated-normal proposals in-kernel (smcdet_amd/csrc/mh_kernel.hip) and
the prior kernels evaluate the truncated Pareto density on device.
"""
from __future__ import annotations

import math

import torch
from torch.distributions import Distribution, Normal


class DiscreteUniform(Distribution):
    def __init__(self, low, high):
        self.low = low
        self.high = high
        super().__init__(validate_args=False)

    def sample(self, sample_shape=torch.Size()):
        return torch.randint(self.low, self.high + 1, tuple(sample_shape))

    def log_prob(self, value):
        in_support = (value >= self.low) & (value <= self.high)
        prob = 1.0 / (self.high - self.low + 1)
        return torch.where(in_support, torch.log(torch.tensor(prob, device=value.device)),
                           torch.tensor(float("-inf"), device=value.device))


class TruncatedDiagonalMVN(Distribution):
    """Normal(mu, sigma) truncated to the box [lb, ub], per dimension."""

    def __init__(self, mu, sigma, lb, ub):
        super().__init__(validate_args=False)
        self.dim = mu.size()
        self.lb = lb
        self.ub = ub
        self.base_dist = Normal(mu, sigma, validate_args=False)
        prob_in_box_hw = self.base_dist.cdf(self.ub) - self.base_dist.cdf(self.lb)
        self.log_prob_in_box = prob_in_box_hw.log().nan_to_num()

    def sample(self, shape=None, u=None):
        if shape is None:
            shape = tuple(self.dim)
        p = torch.rand(shape, device=self.base_dist.loc.device) if u is None else u
        p = p.clamp(min=1e-6, max=1.0 - 1e-6)
        p_tilde = self.base_dist.cdf(self.lb) + p * (self.log_prob_in_box.exp())
        x = self.base_dist.icdf(p_tilde.clamp(min=1e-6, max=1.0 - 1e-6))
        return x.clamp(min=self.lb, max=self.ub)

    def log_prob(self, value):
        if not ((value >= self.lb).all() and (value <= self.ub).all()):
            raise AssertionError("value outside the truncation box")
        return self.base_dist.log_prob(value) - self.log_prob_in_box

    def cdf(self, value):
        cdf_at_val = self.base_dist.cdf(value)
        cdf_at_lb = self.base_dist.cdf(self.lb)
        log_cdf = (cdf_at_val - cdf_at_lb + 1e-9).log().sum(-1) - self.log_prob_in_box
        return log_cdf.exp()


class TruncatedPareto(Distribution):
    """Bounded Pareto(alpha) on [lower, upper]."""

    def __init__(self, alpha, lower, upper):
        self.alpha = torch.tensor(alpha)
        self.lower = torch.tensor(lower)
        self.upper = torch.tensor(upper)
        a, L, U = float(alpha), float(lower), float(upper)
        self.logpdf_norm_const = torch.tensor(
            math.log(a) + a * math.log(L) + a * math.log(U) - math.log(U ** a - L ** a))

    def sample(self, shape=(), device=None, u=None):
        """u: injected uniforms of `shape` (as TruncatedDiagonalMVN.sample's),
        else torch.rand draws them."""
        device = device if device is not None else torch.get_default_device()
        unif = torch.rand(tuple(shape), device=device) if u is None else u.to(device)
        a, L, U = self.alpha.to(device), self.lower.to(device), self.upper.to(device)
        numerator = U ** a - unif * (U ** a) + unif * (L ** a)
        denominator = (L ** a) * (U ** a)
        return (numerator / denominator) ** (-1 / a)

    def log_prob(self, value):
        if not ((value >= self.lower.to(value.device)).all()
                and (value <= self.upper.to(value.device)).all()):
            raise AssertionError("value outside [lower, upper]")
        return (self.logpdf_norm_const.to(value.device)
                - (self.alpha.to(value.device) + 1) * value.log())
