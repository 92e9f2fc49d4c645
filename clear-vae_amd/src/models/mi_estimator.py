"""MI upper-bound estimators with the reference's modules and method names
(code/src/models/mi_estimator.py).  CLUBSample and L1OutUB — the two estimators the CLEAR-MIM
trainer instantiates — run on libclearvae_hip.so: forward / learning_loss /
their gradients are HIP kernels (cvhip.autograd.MIUpperBoundFn / LearningLossFn).

CLUB, CLUBMean, VarUB and InfoNCE are never instantiated by a CLEAR trainer, factory, script or
demo; they are kept importable as plain PyTorch tensor code.
"""

from __future__ import annotations

import torch
import torch.nn as nn
from torch import Tensor

from cvhip import autograd as _ag
from cvhip._lib import MI_CLUBSAMPLE, MI_L1OUT


def _q_nets(x_dim, y_dim, hidden_size):
    """p_mu and p_logvar MLPs of q(y|x) (mi_estimator.py:111-122)."""
    h = hidden_size // 2
    p_mu = nn.Sequential(nn.Linear(x_dim, h), nn.ReLU(), nn.Linear(h, y_dim))
    p_logvar = nn.Sequential(nn.Linear(x_dim, h), nn.ReLU(), nn.Linear(h, y_dim), nn.Tanh())
    return p_mu, p_logvar


class _QEstimator(nn.Module):
    def __init__(self, x_dim, y_dim, hidden_size):
        super().__init__()
        self.p_mu, self.p_logvar = _q_nets(x_dim, y_dim, hidden_size)

    def get_mu_logvar(self, x_samples):
        return self.p_mu(x_samples), self.p_logvar(x_samples)

    def loglikeli(self, x_samples, y_samples):
        if x_samples.device.type == "cuda":
            return -self.learning_loss(x_samples, y_samples)
        mu, logvar = self.get_mu_logvar(x_samples)
        return (-((mu - y_samples) ** 2) / logvar.exp() - logvar).sum(dim=1).mean(dim=0)

    def learning_loss(self, x_samples, y_samples):
        _ag._require_gpu(x_samples, y_samples)
        return _ag.LearningLossFn.apply(x_samples, y_samples, self, *_ag.est_params(self))


class CLUBSample(_QEstimator):
    """Sampled CLUB (mi_estimator.py:108-146); the negative pairs use a device permutation."""

    def forward(self, x_samples, y_samples):
        _ag._require_gpu(x_samples, y_samples)
        return _ag.MIUpperBoundFn.apply(x_samples, y_samples, self, MI_CLUBSAMPLE, *_ag.est_params(self))


class L1OutUB(_QEstimator):
    """Leave-one-out bound with the reference's exact broadcasting semantics (mi_estimator.py:149-198)."""

    def forward(self, x_samples, y_samples):
        _ag._require_gpu(x_samples, y_samples)
        return _ag.MIUpperBoundFn.apply(x_samples, y_samples, self, MI_L1OUT, *_ag.est_params(self))


# ----------------------------------------------------------------------------- not on the hot path


class CLUB(_QEstimator):
    def forward(self, x_samples, y_samples):
        mu, logvar = self.get_mu_logvar(x_samples)
        positive = -((mu - y_samples) ** 2) / 2.0 / logvar.exp()
        negative = -((y_samples.unsqueeze(0) - mu.unsqueeze(1)) ** 2).mean(dim=1) / 2.0 / logvar.exp()
        return (positive.sum(dim=-1) - negative.sum(dim=-1)).mean()


class CLUBMean(nn.Module):
    def __init__(self, x_dim, y_dim, hidden_size=None):
        super().__init__()
        if hidden_size is None:
            self.p_mu = nn.Linear(x_dim, y_dim)
        else:
            self.p_mu = nn.Sequential(nn.Linear(x_dim, int(hidden_size)), nn.ReLU(), nn.Linear(int(hidden_size), y_dim))

    def get_mu_logvar(self, x_samples):
        return self.p_mu(x_samples), 0

    def forward(self, x_samples, y_samples):
        mu, _ = self.get_mu_logvar(x_samples)
        positive = -((mu - y_samples) ** 2) / 2.0
        negative = -((y_samples.unsqueeze(0) - mu.unsqueeze(1)) ** 2).mean(dim=1) / 2.0
        return (positive.sum(dim=-1) - negative.sum(dim=-1)).mean()

    def loglikeli(self, x_samples, y_samples):
        mu, _ = self.get_mu_logvar(x_samples)
        return (-((mu - y_samples) ** 2)).sum(dim=1).mean(dim=0)

    def learning_loss(self, x_samples, y_samples):
        return -self.loglikeli(x_samples, y_samples)


class VarUB(_QEstimator):
    def forward(self, x_samples, y_samples):
        mu, logvar = self.get_mu_logvar(x_samples)
        return 1.0 / 2.0 * (mu**2 + logvar.exp() - 1.0 - logvar).mean()


def logsumexp(x: Tensor, dim: int) -> Tensor:
    """Masked-stable logsumexp (mi_estimator.py:234-242): an all -inf slice gives -inf."""
    m, _ = x.max(dim=dim)
    mask = m == -float("inf")
    s = (x - m.masked_fill(mask, 0).unsqueeze(dim=dim)).exp().sum(dim=dim)
    return s.masked_fill(mask, 1).log() + m.masked_fill(mask, -float("inf"))


class InfoNCE(nn.Module):
    def __init__(self, x_dim, y_dim, hidden_size):
        super().__init__()
        self.F_func = nn.Sequential(
            nn.Linear(x_dim + y_dim, hidden_size), nn.ReLU(), nn.Linear(hidden_size, 1), nn.Softplus()
        )

    def forward(self, x_samples, y_samples):
        n = y_samples.shape[0]
        x_tile = x_samples.unsqueeze(0).repeat((n, 1, 1))
        y_tile = y_samples.unsqueeze(1).repeat((1, n, 1))
        t0 = self.F_func(torch.cat([x_samples, y_samples], dim=-1))
        t1 = self.F_func(torch.cat([x_tile, y_tile], dim=-1))
        return t0.mean() - (t1.logsumexp(dim=1).mean() - torch.tensor(n).log())

    def learning_loss(self, x_samples, y_samples):
        return -self.forward(x_samples, y_samples)
