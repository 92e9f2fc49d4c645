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
# GVAE / ML-VAE (reference vae.py:159-223).  The evidence is segmented by label on the device
# (cvhip.autograd.GroupEvidenceFn -> cv_group_forward / cv_group_evidence_backward); the grouped
# reparameterisation gathers the group rows into group order, samples them with the HIP sampler (so
# noise is consumed in the reference's group-after-group order) and scatters back to batch order.
# The fused trainer step does all of this inside cv_group_forward / cv_group_backward.


def accumulate_group_evidence(mu_c, logvar_c, label_batch, mode: str):
    """(mu_g [m, d], logvar_g [m, d], {label: member indices}) (vae.py:159-190)."""
    _ag._require_gpu(mu_c, logvar_c)
    meta = {}
    mu_g, lv_g = _ag.GroupEvidenceFn.apply(mu_c, logvar_c, label_batch, mode, meta)
    return mu_g, lv_g, meta["groups"]


def groupwise_reparam_each(mu_acc_grp, logvar_acc_grp, g_idx: dict):
    """(z_c [n, d] in batch order, member indices in group order, group size per member) (vae.py:193-223)."""
    _ag._require_gpu(mu_acc_grp, logvar_acc_grp)
    device = mu_acc_grp.device
    idx = [i.to(device) for i in g_idx.values()]
    counts = torch.tensor([len(i) for i in idx], device=device)
    gid = torch.repeat_interleave(torch.arange(len(idx), device=device), counts)
    z_sorted = _ag.SampleFn.apply(mu_acc_grp[gid].contiguous(), logvar_acc_grp[gid].contiguous())
    indices = torch.cat(idx)
    sizes = counts[gid]
    inverse = torch.empty_like(indices)
    inverse[indices] = torch.arange(len(indices), device=device)
    return z_sorted[inverse], indices, sizes
