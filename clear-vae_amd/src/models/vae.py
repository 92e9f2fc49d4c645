"""VAE / VAE64 with the reference's module tree, state_dict keys and init RNG order
(code/src/models/vae.py:7-156), executed by the HIP kernels of libclearvae_hip.so.

The modules stay real ``nn.Conv2d`` / ``nn.ConvTranspose2d`` / ``nn.Linear`` / ``nn.BatchNorm*``
parameter holders (so ``.apply(init_weights)``, ``load_state_dict``, ``requires_grad=False`` freezing
and optimizers behave exactly as with the reference), but ``encode`` / ``decode`` / ``sample`` run
through cvhip.autograd on the device.  There is no CPU path: CPU tensors raise.
"""

from __future__ import annotations

import torch
import torch.nn as nn

from cvhip import autograd as _ag
from cvhip.plan import ensure_arena

# (in, out, kernel, stride, padding[, output_padding]) per layer; channel None = the image channels
_ENC28 = [(None, 32, 3, 2, 1), (32, 64, 3, 2, 1), (64, 128, 3, 2, 1)]
_DEC28 = [(128, 64, 3, 2, 1, 0), (64, 32, 3, 2, 1, 1), (32, None, 3, 2, 1, 1)]
_ENC64 = [(None, 32, 4, 2, 1), (32, 64, 4, 2, 1), (64, 128, 4, 2, 1), (128, 256, 4, 2, 1), (256, 512, 4, 2, 1)]
_DEC64 = [(512, 256, 4, 2, 1, 0), (256, 128, 4, 2, 1, 0), (128, 64, 4, 2, 1, 0), (64, 32, 4, 2, 1, 0),
          (32, None, 4, 2, 1, 0)]
_FEATURES = 2048


def _encoder(table, image_ch):
    layers = []
    for cin, cout, k, s, p in table:
        layers += [nn.Conv2d(image_ch if cin is None else cin, cout, k, s, p), nn.BatchNorm2d(cout), nn.ReLU()]
    return nn.Sequential(*layers, nn.Flatten())


def _decoder(table, z_total, image_ch, unflat):
    layers = [nn.Linear(z_total, _FEATURES), nn.BatchNorm1d(_FEATURES), nn.ReLU(), nn.Unflatten(1, unflat)]
    for i, (cin, cout, k, s, p, op) in enumerate(table):
        c = image_ch if cout is None else cout
        last = i == len(table) - 1
        layers += [nn.ConvTranspose2d(cin, c, k, s, p, op), nn.BatchNorm2d(c), nn.Sigmoid() if last else nn.ReLU()]
    return nn.Sequential(*layers)


class VAE(nn.Module):
    """28x28 CLEAR-VAE (reference code/src/models/vae.py:7-102)."""

    _enc_table, _dec_table, _unflat = _ENC28, _DEC28, (128, 4, 4)

    def __init__(self, total_z_dim, in_channel: int = 1, group_mode: str | None = None) -> None:
        super().__init__()
        self.mode = group_mode
        self.z_dim = int(total_z_dim / 2)
        self._build(VAE._enc_table, VAE._dec_table, VAE._unflat, in_channel)

    def _build(self, enc_table, dec_table, unflat, in_channel):
        # same construction order as the reference: encoder, 4 heads, decoder (init RNG parity)
        self.encoder = _encoder(enc_table, in_channel)
        self.mu_c = nn.Linear(_FEATURES, self.z_dim)
        self.logvar_c = nn.Linear(_FEATURES, self.z_dim)
        self.mu_s = nn.Linear(_FEATURES, self.z_dim)
        self.logvar_s = nn.Linear(_FEATURES, self.z_dim)
        self.decoder = _decoder(dec_table, self.z_dim * 2, in_channel, unflat)

    # -- HIP plumbing --------------------------------------------------------------------------
    def _arena(self):
        return ensure_arena(self)

    def encode(self, x):
        self._arena()
        _ag._require_gpu(x)
        return _ag.EncodeFn.apply(x, self, *_ag.encoder_params(self))

    def decode(self, z):
        self._arena()
        _ag._require_gpu(z)
        return _ag.DecodeFn.apply(z, self, *_ag.decoder_params(self))

    def sample(self, mu, logvar):
        """Reparameterization (vae.py:56-60): eps from the device Philox stream (cvhip.rng)."""
        _ag._require_gpu(mu, logvar)
        return _ag.SampleFn.apply(mu, logvar)

    def generate(self, mu_c, logvar_c, mu_s, logvar_s, g_dict: dict | None = None, explicit=False):
        if g_dict is None:
            z_c = self.sample(mu_c, logvar_c)
        else:
            z_c, _, _ = groupwise_reparam_each(mu_c, logvar_c, g_dict)
        z_s = self.sample(mu_s, logvar_s)
        z = torch.cat([z_c, z_s], dim=-1)
        xhat = self.decode(z)
        return (xhat, z) if explicit else xhat

    def forward(self, x, label=None, explicit=False) -> tuple:
        mu_c, logvar_c, mu_s, logvar_s = self.encode(x)
        g_dict = None
        if label is not None:
            mu_c, logvar_c, g_dict = accumulate_group_evidence(mu_c, logvar_c, label, mode=self.mode)
        latent_params = {"mu_c": mu_c, "logvar_c": logvar_c, "mu_s": mu_s, "logvar_s": logvar_s}
        if explicit:
            xhat, z = self.generate(mu_c, logvar_c, mu_s, logvar_s, g_dict, True)
            return xhat, latent_params, z
        return self.generate(mu_c, logvar_c, mu_s, logvar_s, g_dict, False), latent_params


class VAE64(VAE):
    """64x64 CLEAR-VAE (reference code/src/models/vae.py:105-156).  Like the reference, the 28x28
    modules are built first and then replaced, so the initial weights consume the same RNG stream."""

    def __init__(self, total_z_dim, in_channel: int = 3, group_mode: str | None = None) -> None:
        super().__init__(total_z_dim, in_channel, group_mode)
        self.z_dim = int(total_z_dim / 2)
        self._build(_ENC64, _DEC64, (512, 2, 2), in_channel)


# ----------------------------------------------------------------------------- group evidence
# GVAE / ML-VAE baselines (reference vae.py:159-223).  Outside the CLEAR hot path (SURVEY 2, row
# 1b): kept as PyTorch tensor code on the device so the baseline trainers still import and run.


def accumulate_group_evidence(mu_c, logvar_c, label_batch, mode: str):
    device = mu_c.device
    groups = label_batch.unique(sorted=True)
    mu_acc = torch.zeros(len(groups), mu_c.size(1), device=device)
    lv_acc = torch.zeros(len(groups), logvar_c.size(1), device=device)
    group_idx = {}
    for i, g in enumerate(groups):
        gl = g.item()
        sel = label_batch.eq(gl)
        group_idx[gl] = sel.nonzero().view(-1)
        if mode == "MLVAE":
            inv = -logvar_c[sel, :]
            lse = inv.logsumexp(dim=0)
            mu_acc[i] = (mu_c[sel, :] * inv.exp()).sum(dim=0) * torch.exp(-lse)
            lv_acc[i] = -lse
        elif mode == "GVAE":
            mu_acc[i] = mu_c[sel, :].mean(dim=0)
            lv_acc[i] = logvar_c[sel, :].logsumexp(dim=0) - sel.sum().log()
        else:
            raise NotImplementedError("only support using MLVAE or GVAE")
    return mu_acc, lv_acc, group_idx


def groupwise_reparam_each(mu_acc_grp, logvar_acc_grp, g_idx: dict):
    device = mu_acc_grp.device
    std = torch.exp(0.5 * logvar_acc_grp)
    z_grps, indices, sizes = [], [], []
    for i, (g, idx) in enumerate(g_idx.items()):
        n = len(idx)
        eps = torch.randn(n, std.size(1)).to(device)
        z_grps.append(mu_acc_grp[i][None, :] + eps * std[i][None, :])
        indices.append(idx)
        sizes.append(torch.ones_like(idx) * n)
    z_grps = torch.cat(z_grps, dim=0)
    indices = torch.cat(indices, dim=0)
    sizes = torch.cat(sizes, dim=0)
    inverse = torch.zeros_like(indices)
    inverse[indices] = torch.arange(len(indices)).to(indices.device)
    return z_grps[inverse], indices, sizes
