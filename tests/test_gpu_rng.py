"""The production path's randomness, which every parity test replaces by injection:

  * the reparameterisation noise eps (cv_reparam / the fused step's Philox4x32-10 draw), which replaces
    torch.randn_like in VAE.sample (/root/reference/code/src/models/vae.py:56-60): recovered from the step's
    own heads and z as eps = (z - mu) / exp(logvar / 2), it must be standard normal (mean, variance,
    Kolmogorov-Smirnov), eps_c independent of eps_s and of the other latent dimensions, and fresh at every step,
    the eager first step and every replay of the captured graph alike;
  * the CLUB-S permutation (mi_perm_kernel: Philox keys + a bitonic sort in LDS), which replaces torch.randperm
    at /root/reference/code/src/models/mi_estimator.py:138: a bijection of range(n) at every step (ragged and
    power-of-two n), its inverse consistent, and a fresh permutation per step.

Statistical bars are 5 sigma of the sample size (false-alarm probability < 1e-6 per check)."""

import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _trainer(mode, n_est=None):
    from src.utils.trainer_utils import get_clearmimvae_trainer, get_clearvae_trainer

    torch.manual_seed(0)
    if mode == "clear":
        return get_clearvae_trainer(beta=1 / 8, ps=True, vae_lr=5e-4, z_dim=16, alpha=100, temperature=0.1,
                                    device="cuda", verbose_period=10**9)
    return get_clearmimvae_trainer(beta=1 / 8, mi_estimator="CLUBSample", la=3.0, vae_lr=5e-4, mi_estimator_lr=2e-3,
                                   z_dim=16, alpha=100, temperature=0.1, device="cuda", verbose_period=10**9)


def _eps(ws, d):
    h = ws.heads.double().cpu()
    z = ws.z.double().cpu()
    ec = (z[:, :d] - h[:, :d]) / torch.exp(0.5 * h[:, d:2 * d])
    es = (z[:, d:] - h[:, 2 * d:3 * d]) / torch.exp(0.5 * h[:, 3 * d:])
    return ec.numpy(), es.numpy()


def test_reparam_noise_is_fresh_standard_normal():
    from scipy import stats

    from cvhip import rng
    from cvhip.engine import ClearStep

    n = 2048
    tr = _trainer("clear")
    eng = ClearStep.build(tr, "clear")
    assert eng is not None
    rng.clear_injections()
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.rand(n, 1, 28, 28, generator=g, device="cuda")
    L = torch.randint(0, 10, (n,), generator=g, device="cuda")
    d = eng.spec.d
    draws = []
    for step in range(4):  # eager, capture + replay, replay, replay
        eng.step(X, L)
        torch.cuda.synchronize()
        draws.append(_eps(eng.last_workspace(n), d))
    assert "graphs" in eng.graphs[n]
    for ec, es in draws:
        for e in (ec, es):
            v = e.reshape(-1)
            N = v.size
            assert np.isfinite(v).all()
            assert abs(v.mean()) < 5 / math.sqrt(N), v.mean()
            assert abs(v.var() - 1) < 5 * math.sqrt(2 / N), v.var()
            assert stats.kstest(v, "norm").pvalue > 1e-6
        # eps_c independent of eps_s, and the latent dimensions of one draw of each other
        c = np.corrcoef(np.concatenate([ec, es], axis=1), rowvar=False)
        off = c[~np.eye(2 * d, dtype=bool)]
        assert np.abs(off).max() < 5 / math.sqrt(n), np.abs(off).max()
    # fresh noise at every step (eager -> first replay -> later replays)
    for (a, _), (b, _) in zip(draws, draws[1:]):
        assert not np.array_equal(a, b)
        r = np.corrcoef(a.reshape(-1), b.reshape(-1))[0, 1]
        assert abs(r) < 5 / math.sqrt(a.size), r


def _mi_perm(ws, n):
    """perm / invperm of the CLUB-S forward in the step's MI workspace (cv_mi.hip mi_work layout)."""
    nb, fp, gsz = 64, 2 + 128, 4 * 64 * 64 + 256
    off = 4 * 64 * 8 + nb * fp * 8 + nb * 8 + 64 + nb * gsz * 4
    raw = ws.mi_work.view(torch.int32).cpu().numpy()
    perm = raw[off // 4: off // 4 + n].copy()
    inv = raw[off // 4 + n: off // 4 + 2 * n].copy()
    return perm, inv


@pytest.mark.parametrize("n", [256, 1000])
def test_clubsample_device_permutation_is_fresh_bijection(n):
    from cvhip import rng
    from cvhip.engine import ClearStep

    tr = _trainer("mim")
    eng = ClearStep.build(tr, "mim")
    assert eng is not None
    rng.clear_injections()
    g = torch.Generator(device="cuda").manual_seed(4)
    X = torch.rand(n, 1, 28, 28, generator=g, device="cuda")
    L = torch.randint(0, 10, (n,), generator=g, device="cuda")
    perms = []
    fixed = 0
    for step in range(4):
        eng.step(X, L)
        torch.cuda.synchronize()
        perm, inv = _mi_perm(eng.last_workspace(n), n)
        assert np.array_equal(np.sort(perm), np.arange(n)), "not a permutation"
        assert np.array_equal(inv[perm], np.arange(n)), "inverse inconsistent"
        fixed += int((perm == np.arange(n)).sum())
        perms.append(perm)
    assert "graphs" in eng.graphs[n]
    for a, b in zip(perms, perms[1:]):
        assert not np.array_equal(a, b), "same permutation on consecutive steps"
    # a uniform permutation has 1 fixed point on average (Poisson(1)): over 4 draws, far below 20
    assert fixed < 20, fixed
    # and is not the identity or a shift: positions move by about n/3 on average
    assert np.mean([np.abs(p - np.arange(n)).mean() for p in perms]) > n / 4
