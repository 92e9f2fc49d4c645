"""ORACLE — test / measurement infrastructure only (never imported by the product path).

The CPU baseline of bench.py: the reference's training loop restated with its own step composition, so its
host-core speed stands in for the reference's CPU path on the GPU box (where /root/reference does not
exist).  Where oracle/cpu_ref.py is a functional fp64 restatement for parity, this module mirrors how the
reference *executes* a step, which is what its speed depends on:

  * nn.Module model (nn.Sequential Conv/BN/ReLU encoder, 4 Linear heads, Linear/BN1d/Unflatten/ConvT
    decoder), the layer tables of cpu_ref (reference code/src/models/vae.py:15-46, 113-156), eps drawn
    with torch.randn_like inside the forward (vae.py:56-60);
  * vae_loss through F.mse_loss(reduction="none") and per-sample sums (losses.py:36-50);
  * contrastive_loss with float pair masks, boolean index_put fills of the diagonal and of the negatives,
    a TorchScript masked logsumexp and the boolean-indexed finite-row mean (losses.py:87-137);
  * CLUBSample with torch.randperm on the CPU generator (mi_estimator.py:108-146);
  * the trainer step order of CLEARVAETrainer._train (trainer.py:447-492) / ClearMIMVAETrainer._train
    (trainer.py:842-897): zero_grad, forward, losses, backward, torch.optim.Adam, annealer, and the
    per-step float() reads of the progress-bar postfix.

Calibration (development container, 8 threads, synthetic U[0,1) batches): see DESIGN.md §7 — this loop and
the real reference's CLEARVAETrainer._train are timed side by side by tests/golden/calibrate_cpu.py.
"""

from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle.cpu_ref import DEC, ENC, UNFLAT


class RefVAE(nn.Module):
    """Same module tree (and state_dict keys) as the reference VAE / VAE64."""

    def __init__(self, arch: str, total_z_dim: int, in_channel: int):
        super().__init__()
        self.z_dim = total_z_dim // 2
        enc = []
        for cin, cout, k, s, p in ENC[arch]:
            enc += [nn.Conv2d(in_channel if cin is None else cin, cout, k, s, p), nn.BatchNorm2d(cout), nn.ReLU()]
        self.encoder = nn.Sequential(*enc, nn.Flatten())
        feat = 2048
        self.mu_c, self.logvar_c, self.mu_s, self.logvar_s = (nn.Linear(feat, self.z_dim) for _ in range(4))
        dec = [nn.Linear(2 * self.z_dim, feat), nn.BatchNorm1d(feat), nn.ReLU(), nn.Unflatten(1, UNFLAT[arch])]
        for j, (cin, cout, k, s, p, op) in enumerate(DEC[arch]):
            cout = in_channel if cout is None else cout
            last = j == len(DEC[arch]) - 1
            dec += [nn.ConvTranspose2d(cin, cout, k, s, p, op), nn.BatchNorm2d(cout), nn.Sigmoid() if last else nn.ReLU()]
        self.decoder = nn.Sequential(*dec)

    def forward(self, x, explicit=False):
        h = self.encoder(x)
        mu_c, lv_c, mu_s, lv_s = self.mu_c(h), self.logvar_c(h), self.mu_s(h), self.logvar_s(h)
        z = torch.cat([mu_c + torch.randn_like(lv_c) * torch.exp(0.5 * lv_c),
                       mu_s + torch.randn_like(lv_s) * torch.exp(0.5 * lv_s)], dim=-1)
        lp = {"mu_c": mu_c, "logvar_c": lv_c, "mu_s": mu_s, "logvar_s": lv_s}
        xhat = self.decoder(z)
        return (xhat, lp, z) if explicit else (xhat, lp)


class RefCLUBSample(nn.Module):
    def __init__(self, d: int, hidden: int):
        super().__init__()
        self.p_mu = nn.Sequential(nn.Linear(d, hidden // 2), nn.ReLU(), nn.Linear(hidden // 2, d))
        self.p_logvar = nn.Sequential(nn.Linear(d, hidden // 2), nn.ReLU(), nn.Linear(hidden // 2, d), nn.Tanh())

    def forward(self, x, y):
        mu, lv = self.p_mu(x), self.p_logvar(x)
        idx = torch.randperm(x.shape[0]).long()
        pos = -((mu - y) ** 2) / lv.exp()
        neg = -((mu - y[idx]) ** 2) / lv.exp()
        return (pos.sum(dim=-1) - neg.sum(dim=-1)).mean() / 2.0

    def learning_loss(self, x, y):
        mu, lv = self.p_mu(x), self.p_logvar(x)
        return -((-((mu - y) ** 2) / lv.exp() - lv).sum(dim=1).mean(dim=0))


def _per_sample_mean(t):
    return t.sum(dim=list(range(t.dim()))[1:]).mean()


def vae_loss(xhat, x, mu_c, mu_s, logvar_c, logvar_s):
    rec = _per_sample_mean(F.mse_loss(xhat, x, reduction="none"))
    kl_c = -0.5 * _per_sample_mean(1 + logvar_c - mu_c.pow(2) - logvar_c.exp())
    kl_s = -0.5 * _per_sample_mean(1 + logvar_s - mu_s.pow(2) - logvar_s.exp())
    return rec, kl_c, kl_s


@torch.jit.script
def _lse(x: torch.Tensor, dim: int) -> torch.Tensor:
    m, _ = x.max(dim=dim)
    dead = m == -float("inf")
    s = (x - m.masked_fill_(dead, 0).unsqueeze(dim=dim)).exp().sum(dim=dim)
    return s.masked_fill_(dead, 1).log() + m.masked_fill_(dead, -float("inf"))


def contrastive_loss(mu, label, temperature, ps=False):
    """cosine similarity branch (the factories' sim_fn, trainer_utils.py:104,189)"""
    pair = (label[None, :] != label[:, None]).float() if ps else (label[None, :] == label[:, None]).float()
    sim = F.cosine_similarity(mu[None, :, :], mu[:, None, :], dim=-1)
    n = sim.shape[0]
    sim[torch.eye(n).bool()] = float("-inf")
    pos = pair * sim
    pos[pair == 0] = float("-inf")
    losses = -_lse(pos / temperature, 1) + _lse(sim / temperature, 1)
    return losses[torch.isfinite(losses)].mean()


class RefLoop:
    """One process's CLEAR-VAE / CLEAR-MIM (CLUB-S) training loop on torch-CPU."""

    def __init__(self, arch, z, in_ch, mode, hp, seed=0):
        torch.manual_seed(seed)
        self.vae = RefVAE(arch, z, in_ch)
        self.opt = torch.optim.Adam(self.vae.parameters(), lr=hp["vae_lr"])
        self.mode, self.hp, self.t = mode, hp, 0
        if mode == "mim":
            self.est = RefCLUBSample(z // 2, z)
            self.est_opt = torch.optim.Adam(self.est.parameters(), lr=hp["mi_lr"])

    def _w(self):  # LogisticAnnealer(loc=0, scale=1)
        return self.hp["beta"] / (1 + math.exp(-self.t))

    def step(self, X, label):
        hp, vae, d = self.hp, self.vae, self.vae.z_dim
        vae.train()
        if self.mode == "clear":
            self.opt.zero_grad()
            xhat, lp = vae(X)
            rec, kl_c, kl_s = vae_loss(xhat, X, **lp)
            c = contrastive_loss(lp["mu_c"], label, hp["temperature"])
            s = contrastive_loss(lp["mu_s"], label, hp["temperature"], ps=hp["ps"])
            if not hp["ps"]:
                s = -s
            w = self._w()
            loss = rec + w * kl_c + w * kl_s + hp["alpha"] * c + hp["alpha"] * s
            loss.backward()
            self.opt.step()
            self.t += 1
            return [float(rec), float(kl_c), float(kl_s), float(c), float(s)]
        xhat, lp, z = vae(X, explicit=True)
        self.opt.zero_grad()
        rec, kl_c, kl_s = vae_loss(xhat, X, **lp)
        c = contrastive_loss(lp["mu_c"], label, hp["temperature"])
        mi = self.est(z[:, :d], z[:, d:])
        w = self._w()
        loss = rec + w * kl_c + w * kl_s + hp["alpha"] * c + hp["la"] * mi
        mi_v = float(mi)
        loss.backward()
        self.opt.step()
        self.t += 1
        learn = []
        for _ in range(5):
            _, _, z2 = vae(X, explicit=True)
            z2 = z2.detach()
            ll = self.est.learning_loss(z2[:, :d], z2[:, d:])
            self.est_opt.zero_grad()
            ll.backward()
            self.est_opt.step()
            learn.append(float(ll))
        return [float(rec), float(kl_c), float(kl_s), float(c), mi_v] + learn
