"""ORACLE — test infrastructure only (never imported by the product path).

A functional, CPU restatement of the reference's CLEAR-VAE hot path (scotsun/clear-vae @ code/src),
written against torch.nn.functional so that it runs in fp32 or fp64 on the host.  It restates:

  VAE / VAE64 forward          code/src/models/vae.py:15-46, 48-102, 113-156
  vae_loss                     code/src/losses.py:36-50
  pairwise similarities        code/src/losses.py:53-84
  logsumexp / snn_loss         code/src/losses.py:87-95, 129-137
  contrastive_loss             code/src/losses.py:98-126
  CLUBSample / L1OutUB         code/src/models/mi_estimator.py:108-198
  factor discriminator, factor_shuffling, CLEAR-TC step
                               code/src/utils/trainer_utils.py:133-138, code/src/trainer.py:573-699
  LogisticAnnealer             code/src/trainer.py:22-38
  CLEARVAETrainer step         code/src/trainer.py:447-484
  ClearMIMVAETrainer step      code/src/trainer.py:842-888
  ClearTCVAETrainer step       code/src/trainer.py:648-699
  GVAE / ML-VAE group evidence code/src/models/vae.py:159-223
  HierarchicalVAETrainer step  code/src/trainer.py:322-353
with the reparameterisation noise and the CLUB-S permutation passed in explicitly.
Gradients come from torch autograd on the CPU.

Pinning: tests/golden/*.npz hold outputs of the REAL reference (imported from /root/reference in the
development container by tests/golden/gen_golden.py, fp64, same deterministic weights / inputs /
noise); tests/test_oracle_golden.py checks this restatement against them.  Only tests/, the
__graft_entry__.smoke() check and bench.py's cpu_baseline leg use this module.
"""

from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------- architecture tables
# (in, out, k, s, p[, op]); None = image channels.   vae.py:15-46 (VAE) and :113-156 (VAE64)
ENC = {"VAE": [(None, 32, 3, 2, 1), (32, 64, 3, 2, 1), (64, 128, 3, 2, 1)],
       "VAE64": [(None, 32, 4, 2, 1), (32, 64, 4, 2, 1), (64, 128, 4, 2, 1), (128, 256, 4, 2, 1),
                 (256, 512, 4, 2, 1)]}
DEC = {"VAE": [(128, 64, 3, 2, 1, 0), (64, 32, 3, 2, 1, 1), (32, None, 3, 2, 1, 1)],
       "VAE64": [(512, 256, 4, 2, 1, 0), (256, 128, 4, 2, 1, 0), (128, 64, 4, 2, 1, 0), (64, 32, 4, 2, 1, 0),
                 (32, None, 4, 2, 1, 0)]}
UNFLAT = {"VAE": (128, 4, 4), "VAE64": (512, 2, 2)}
IMAGE = {"VAE": 28, "VAE64": 64}


def state_keys(arch: str, z_total: int, in_ch: int):
    """state_dict keys/shapes of the reference module tree (parameters and BN buffers)."""
    d = z_total // 2
    out = []
    i = 0
    for cin, cout, k, s, p in ENC[arch]:
        cin = in_ch if cin is None else cin
        out += [(f"encoder.{i}.weight", (cout, cin, k, k)), (f"encoder.{i}.bias", (cout,))]
        out += [(f"encoder.{i + 1}.{n}", (cout,)) for n in ("weight", "bias", "running_mean", "running_var")]
        out += [(f"encoder.{i + 1}.num_batches_tracked", ())]
        i += 3
    for h in ("mu_c", "logvar_c", "mu_s", "logvar_s"):
        out += [(f"{h}.weight", (d, 2048)), (f"{h}.bias", (d,))]
    out += [("decoder.0.weight", (2048, 2 * d)), ("decoder.0.bias", (2048,))]
    out += [(f"decoder.1.{n}", (2048,)) for n in ("weight", "bias", "running_mean", "running_var")]
    out += [("decoder.1.num_batches_tracked", ())]
    i = 4
    for cin, cout, k, s, p, op in DEC[arch]:
        cout = in_ch if cout is None else cout
        out += [(f"decoder.{i}.weight", (cin, cout, k, k)), (f"decoder.{i}.bias", (cout,))]
        out += [(f"decoder.{i + 1}.{n}", (cout,)) for n in ("weight", "bias", "running_mean", "running_var")]
        out += [(f"decoder.{i + 1}.num_batches_tracked", ())]
        i += 3
    return out


def det_state(arch: str, z_total: int, in_ch: int, seed: int = 0) -> dict:
    """Deterministic, platform-independent weights (numpy PCG64): U(-b, b) with the PyTorch default
    bound b = 1/sqrt(fan_in) for conv/linear, BN weight U(0.5, 1.5), BN bias U(-0.1, 0.1), running
    stats at their defaults.  Used by the golden generator AND the tests so no weights are stored."""
    rng = np.random.default_rng(seed)
    sd = {}
    for name, shape in state_keys(arch, z_total, in_ch):
        if name.endswith("num_batches_tracked"):
            sd[name] = np.array(0, dtype=np.int64)
            continue
        if name.endswith("running_mean"):
            sd[name] = np.zeros(shape)
            continue
        if name.endswith("running_var"):
            sd[name] = np.ones(shape)
            continue
        parts = name.split(".")
        is_bn = False
        if parts[0] in ("encoder", "decoder"):
            idx = int(parts[1])
            layer_kind = _layer_kind(arch, parts[0], idx)
            is_bn = layer_kind == "bn"
        if is_bn:
            sd[name] = rng.uniform(0.5, 1.5, shape) if parts[-1] == "weight" else rng.uniform(-0.1, 0.1, shape)
            continue
        wname = ".".join(parts[:-1]) + ".weight"
        wshape = dict(state_keys(arch, z_total, in_ch))[wname]
        if len(wshape) == 4:
            is_t = parts[0] == "decoder"
            fan_in = (wshape[0] if is_t else wshape[1]) * wshape[2] * wshape[3]
            if is_t:  # ConvTranspose2d fan_in = weight.size(1) * k * k in torch's init
                fan_in = wshape[1] * wshape[2] * wshape[3]
        else:
            fan_in = wshape[1]
        b = 1.0 / math.sqrt(fan_in)
        sd[name] = rng.uniform(-b, b, shape)
    return sd


def _layer_kind(arch, part, idx):
    if part == "encoder":
        return ["conv", "bn", "relu"][idx % 3]
    if idx == 0:
        return "linear"
    if idx == 1:
        return "bn"
    if idx < 4:
        return "other"
    return ["conv", "bn", "act"][(idx - 4) % 3]


def det_inputs(n: int, in_ch: int, hw: int, z_total: int, n_labels: int, seed: int = 1):
    """x ~ U[0,1) NCHW, labels, eps_c, eps_s ~ N(0,1), CLUB-S permutation (numpy PCG64)."""
    rng = np.random.default_rng(seed)
    x = rng.random((n, in_ch, hw, hw))
    label = rng.integers(0, n_labels, size=n).astype(np.int64)
    d = z_total // 2
    eps_c = rng.standard_normal((n, d))
    eps_s = rng.standard_normal((n, d))
    perm = rng.permutation(n).astype(np.int64)
    return x, label, eps_c, eps_s, perm


def det_mlp(d: int, hidden_size: int, seed: int = 2) -> dict:
    """Deterministic estimator weights (mi_estimator.py:111-122 layout, Linear bound 1/sqrt(fan_in))."""
    rng = np.random.default_rng(seed)
    h = hidden_size // 2
    out = {}
    for net in ("p_mu", "p_logvar"):
        b1 = 1.0 / math.sqrt(d)
        out[f"{net}.0.weight"] = rng.uniform(-b1, b1, (h, d))
        out[f"{net}.0.bias"] = rng.uniform(-b1, b1, (h,))
        b2 = 1.0 / math.sqrt(h)
        out[f"{net}.2.weight"] = rng.uniform(-b2, b2, (d, h))
        out[f"{net}.2.bias"] = rng.uniform(-b2, b2, (d,))
    return out


def det_disc(z_total: int, seed: int = 3) -> dict:
    """Deterministic factor-discriminator weights: nn.Sequential(Linear(z, z), ReLU, Linear(z, 1), Sigmoid)
    (trainer_utils.py:133-138), Linear bound 1/sqrt(fan_in)."""
    rng = np.random.default_rng(seed)
    b = 1.0 / math.sqrt(z_total)
    return {"0.weight": rng.uniform(-b, b, (z_total, z_total)), "0.bias": rng.uniform(-b, b, (z_total,)),
            "2.weight": rng.uniform(-b, b, (1, z_total)), "2.bias": rng.uniform(-b, b, (1,))}


# ----------------------------------------------------------------------------- functional model


def to_torch(sd: dict, dtype=torch.float64, requires_grad=True) -> dict:
    out = {}
    for k, v in sd.items():
        t = torch.as_tensor(np.asarray(v))
        if k.endswith("num_batches_tracked"):
            out[k] = t.clone()
            continue
        t = t.to(dtype).clone()
        if requires_grad and not (k.endswith("running_mean") or k.endswith("running_var")):
            t.requires_grad_(True)
        out[k] = t
    return out


def _bn(x, P, prefix, train):
    rm, rv = P[prefix + ".running_mean"], P[prefix + ".running_var"]
    out = F.batch_norm(x, rm, rv, P[prefix + ".weight"], P[prefix + ".bias"], training=train, momentum=0.1,
                       eps=1e-5)
    if train:
        P[prefix + ".num_batches_tracked"] += 1
    return out


def _relu(h, masks, key):
    """ReLU, or with masks[key] given (a 0/1 tensor of h's shape) the ReLU with its activity pattern pinned:
    h * mask.  Pinning the pattern a device forward chose removes the knife-edge elements whose BN output
    is within rounding of 0 from a gradient comparison (tests/test_gpu_maskpinned.py); away from such
    elements it is the same function, so the pinned gradient is the ReLU's."""
    if masks is not None and key in masks:
        return h * masks[key].to(h.dtype)
    return F.relu(h)


def _r16(t):
    """Round to bf16 (nearest even) and back: an operand as the bf16 MFMA path stages it."""
    return t.to(torch.bfloat16).to(t.dtype)


class _Bf16Conv(torch.autograd.Function):
    """conv2d / conv_transpose2d with the contraction operands rounded to bf16 where the HIP GEMM core rounds
    them under precision="bf16" (cv_gemm_tile.inc `store`: after the fp32 BN transform, before the LDS image):
    forward the input activation and the weight; backward the incoming gradient (after the BN backward) in
    both the data and the weight contraction, together with the weight resp. the input activation.  The
    contraction itself stays exact here (fp64 or fp32 accumulation).  Bias gradient: the unrounded sum."""

    @staticmethod
    def forward(ctx, h, w, b, s, p, op, transposed):
        hr, wr = _r16(h), _r16(w)
        ctx.save_for_backward(hr, wr)
        ctx.cfg = (s, p, op, transposed, b is not None)
        return _Bf16Conv._conv(hr, wr, s, p, op, transposed) + (0 if b is None else b.view(1, -1, 1, 1))

    @staticmethod
    def _conv(h, w, s, p, op, transposed):
        if transposed:
            return F.conv_transpose2d(h, w, None, stride=s, padding=p, output_padding=op)
        return F.conv2d(h, w, None, stride=s, padding=p)

    @staticmethod
    def backward(ctx, g):
        hr, wr = ctx.saved_tensors
        s, p, op, transposed, has_b = ctx.cfg
        with torch.enable_grad():
            h_, w_ = hr.detach().requires_grad_(True), wr.detach().requires_grad_(True)
            out = _Bf16Conv._conv(h_, w_, s, p, op, transposed)
            gh, gw = torch.autograd.grad(out, (h_, w_), _r16(g))
        gb = g.sum(dim=(0, 2, 3)) if has_b else None
        return gh, gw, gb, None, None, None, None


def _conv(h, P, name, s, p, op=0, transposed=False, bf16=False):
    """One conv / convT layer; bf16: the GEMM-core operand rounding (_Bf16Conv)."""
    w, b = P[f"{name}.weight"], P[f"{name}.bias"]
    if bf16:
        return _Bf16Conv.apply(h, w, b, s, p, op, transposed)
    if transposed:
        return F.conv_transpose2d(h, w, b, stride=s, padding=p, output_padding=op)
    return F.conv2d(h, w, b, stride=s, padding=p)


def encode(P, x, arch, train=True, masks=None, bf16=False):
    """vae.py:48-50 (encoder 15-26 / 113-130, heads 27-30); masks: _relu.  bf16: the HIP path's precision="bf16"
    arithmetic — every conv but the image-facing first one (an edge kernel, fp32 by design) takes bf16-rounded
    operands (_Bf16Conv); the heads stay fp32 (cvhip/plan.py runs the latent-side linears in fp32)."""
    h = x
    i = 0
    for j, (cin, cout, k, s, p) in enumerate(ENC[arch]):
        h = _conv(h, P, f"encoder.{i}", s, p, bf16=bf16 and j > 0)
        h = _relu(_bn(h, P, f"encoder.{i + 1}", train), masks, f"encoder.{i + 2}")
        i += 3
    h = h.flatten(1)
    return tuple(F.linear(h, P[f"{n}.weight"], P[f"{n}.bias"]) for n in ("mu_c", "logvar_c", "mu_s", "logvar_s"))


def decode(P, z, arch, train=True, masks=None, bf16=False):
    """vae.py:52-54 (decoder 32-46 / 136-156); masks: _relu; bf16: as in encode (every ConvTranspose2d but the
    image-facing last one; the decoder Linear stays fp32)."""
    h = F.linear(z, P["decoder.0.weight"], P["decoder.0.bias"])
    h = _relu(_bn(h, P, "decoder.1", train), masks, "decoder.2")
    h = h.unflatten(1, UNFLAT[arch])
    i = 4
    n_dec = len(DEC[arch])
    for j, (cin, cout, k, s, p, op) in enumerate(DEC[arch]):
        h = _conv(h, P, f"decoder.{i}", s, p, op, True, bf16=bf16 and j < n_dec - 1)
        h = _bn(h, P, f"decoder.{i + 1}", train)
        h = torch.sigmoid(h) if j == n_dec - 1 else _relu(h, masks, f"decoder.{i + 2}")
        i += 3
    return h


def sample(mu, logvar, eps):
    """vae.py:56-60 with explicit eps."""
    return mu + eps * torch.exp(0.5 * logvar)


def vae_forward(P, x, eps_c, eps_s, arch, train=True, masks=None, bf16=False):
    mu_c, lv_c, mu_s, lv_s = encode(P, x, arch, train, masks, bf16)
    z = torch.cat([sample(mu_c, lv_c, eps_c), sample(mu_s, lv_s, eps_s)], dim=-1)
    return decode(P, z, arch, train, masks, bf16), {"mu_c": mu_c, "logvar_c": lv_c, "mu_s": mu_s, "logvar_s": lv_s}, z


# ----------------------------------------------------------------------------- losses


def vae_loss(xhat, x, mu_c, mu_s, logvar_c, logvar_s):
    """losses.py:41-50"""
    def red(t):
        return t.sum(dim=list(range(t.dim()))[1:]).mean()
    rec = red((xhat - x) ** 2)
    kl_c = -0.5 * red(1 + logvar_c - mu_c.pow(2) - logvar_c.exp())
    kl_s = -0.5 * red(1 + logvar_s - mu_s.pow(2) - logvar_s.exp())
    return rec, kl_c, kl_s


def pairwise(sim_fn, mu, logvar):
    """losses.py:53-84 and the dispatch at :111-123"""
    if sim_fn == "cosine":
        return F.cosine_similarity(mu[None, :, :], mu[:, None, :], dim=-1)
    if sim_fn == "l2":
        return -((mu[None, :, :] - mu[:, None, :]) ** 2).sum(dim=-1)
    if sim_fn == "modified_l2":
        var = (0.5 * (logvar[None, :, :] + logvar[:, None, :])).exp()
        return -((mu[None, :, :] - mu[:, None, :]) ** 2 / var).sum(dim=-1)
    if sim_fn == "jeffrey":
        k = mu.shape[1]
        var = logvar.exp()
        t1 = logvar.sum(dim=-1)[None, :] - logvar.sum(dim=-1)[:, None] - k
        t2 = ((mu[None, :, :] - mu[:, None, :]) ** 2 / logvar.exp()).sum(dim=-1)
        t3 = (var[None, :, :] / (var[:, None, :] + 1e-8)).sum(dim=-1)
        kl = 0.5 * (t1 + t2 + t3)
        return -(0.5 * (kl + kl.T))
    if sim_fn == "mahalanobis":
        var = 0.5 * (logvar.exp()[None, :, :] + logvar.exp()[:, None, :])
        return -((mu[None, :, :] - mu[:, None, :]) ** 2 / var).sum(dim=-1)
    raise ValueError("unimplemented similarity measure.")


def logsumexp(x, dim):
    """losses.py:87-95"""
    m, _ = x.max(dim=dim)
    mask = m == -float("inf")
    s = (x - m.masked_fill(mask, 0).unsqueeze(dim)).exp().sum(dim=dim)
    return s.masked_fill(mask, 1).log() + m.masked_fill(mask, -float("inf"))


def snn_loss(sim, pair_mat, temperature):
    """losses.py:129-137 (out-of-place)"""
    n = sim.shape[0]
    eye = torch.eye(n, dtype=torch.bool)
    sim = sim.masked_fill(eye, float("-inf"))
    pos = (pair_mat * sim).masked_fill(pair_mat == 0, float("-inf"))
    return -logsumexp(pos / temperature, dim=1) + logsumexp(sim / temperature, dim=1)


def contrastive_loss(mu, logvar, label, sim_fn, temperature, ps=False):
    """losses.py:98-126"""
    if ps:
        pair = (label[None, :] != label[:, None]).to(mu.dtype)
    else:
        pair = (label[None, :] == label[:, None]).to(mu.dtype)
    losses = snn_loss(pairwise(sim_fn, mu, logvar), pair, temperature)
    return losses[torch.isfinite(losses)].mean()


# ----------------------------------------------------------------------------- large batches
# The reference's contrastive_loss and L1OutUB materialise [N, N, d] / [N, N, N] intermediates; at the batches
# above the HIP kernels' one-workgroup caps (tests/test_gpu_bigbatch.py, N = 8192) those do not fit a host.
# These restate the SAME per-row terms block by block (contrastive) or in closed form (L1Out); each is checked
# against the literal restatement above at small N (tests/test_oracle_golden.py).


def pairwise_rows(sim_fn, mu, logvar, rows):
    """pairwise(sim_fn, mu, logvar)[rows, :] (losses.py:53-84 and :111-123) without the other rows: every
    expression of `pairwise` with its row operand X[:, None] restricted to X[rows][:, None]."""
    mr = mu[rows]
    if sim_fn == "cosine":
        return F.cosine_similarity(mu[None, :, :], mr[:, None, :], dim=-1)
    if sim_fn == "l2":
        return -((mu[None, :, :] - mr[:, None, :]) ** 2).sum(dim=-1)
    lr = logvar[rows]
    if sim_fn == "modified_l2":
        var = (0.5 * (logvar[None, :, :] + lr[:, None, :])).exp()
        return -((mu[None, :, :] - mr[:, None, :]) ** 2 / var).sum(dim=-1)
    if sim_fn == "jeffrey":
        k = mu.shape[1]
        var, vr = logvar.exp(), lr.exp()
        L, Lr = logvar.sum(dim=-1), lr.sum(dim=-1)
        d2 = (mu[None, :, :] - mr[:, None, :]) ** 2
        kl_rj = 0.5 * (L[None, :] - Lr[:, None] - k + (d2 / var[None, :, :]).sum(dim=-1)
                       + (var[None, :, :] / (vr[:, None, :] + 1e-8)).sum(dim=-1))    # kl[i, j], i in rows
        kl_jr = 0.5 * (Lr[:, None] - L[None, :] - k + (d2 / vr[:, None, :]).sum(dim=-1)
                       + (vr[:, None, :] / (var[None, :, :] + 1e-8)).sum(dim=-1))    # kl[j, i]
        return -(0.5 * (kl_rj + kl_jr))
    if sim_fn == "mahalanobis":
        var = 0.5 * (logvar.exp()[None, :, :] + lr.exp()[:, None, :])
        return -((mu[None, :, :] - mr[:, None, :]) ** 2 / var).sum(dim=-1)
    raise ValueError("unimplemented similarity measure.")


def contrastive_rows(mu, logvar, label, sim_fn, temperature, ps, rows):
    """The snn_loss row terms (losses.py:129-137) of `rows`: -LSE(pos/tau) + LSE(sim/tau), diagonal at -inf."""
    sim = pairwise_rows(sim_fn, mu, logvar, rows)
    lab_r = label[rows]
    pair = (label[None, :] != lab_r[:, None]) if ps else (label[None, :] == lab_r[:, None])
    diag = torch.zeros_like(sim, dtype=torch.bool)
    diag[torch.arange(len(rows)), rows] = True
    sim = sim.masked_fill(diag, float("-inf"))
    pos = (pair.to(sim.dtype) * sim).masked_fill(~pair, float("-inf"))
    return -logsumexp(pos / temperature, dim=1) + logsumexp(sim / temperature, dim=1)


def contrastive_loss_blockwise(mu, logvar, label, sim_fn, temperature, ps=False, block=128):
    """contrastive_loss (losses.py:98-126: the mean over the finite rows) accumulated block by block, with the
    gradient w.r.t. mu / logvar (leaves requiring grad) back-propagated per block so only one block's graph is
    alive: returns the loss (a detached scalar); grads land in mu.grad / logvar.grad."""
    n = mu.shape[0]
    blocks = [torch.arange(i, min(n, i + block)) for i in range(0, n, block)]
    with torch.no_grad():
        terms = torch.cat([contrastive_rows(mu, logvar, label, sim_fn, temperature, ps, r) for r in blocks])
    finite = torch.isfinite(terms)
    nf = int(finite.sum())
    loss = terms[finite].sum() / nf
    if mu.requires_grad or (logvar is not None and logvar.requires_grad):
        for r in blocks:
            t = contrastive_rows(mu, logvar, label, sim_fn, temperature, ps, r)
            t[torch.isfinite(t)].sum().div(nf).backward()
    return loss


def l1out_closed(M, x, y):
    """L1OutUB.forward (mi_estimator.py:170-191) in closed form: the [N,N,N] broadcast of all_probs[N,N] with
    diag_mask[N,N,1] makes negative[b,c] = all_probs[b,c] + log((N-1) + e^-20) - log(N-1) (the last log of a
    float32 tensor, :188), and the mean over (b, c) of all_probs is a row sum of O(N d) moments."""
    n = y.shape[0]
    mu, lv = mlp_forward(M, x)
    positive = (-((mu - y) ** 2) / 2.0 / lv.exp() - lv / 2.0).sum(dim=-1)
    sy, sy2 = y.sum(dim=0), (y * y).sum(dim=0)
    rows = (-(sy2[None, :] - 2.0 * mu * sy[None, :] + n * mu ** 2) / 2.0 / lv.exp() - n * lv / 2.0).sum(dim=-1)
    delta = math.log((n - 1) + math.exp(-20.0)) - float((torch.tensor(n) - 1.0).log())
    return positive.mean() - rows.sum() / (n * n) - delta


def mlp_forward(M, x):
    """q(y|x) MLPs (mi_estimator.py:111-127)"""
    mu = F.linear(F.relu(F.linear(x, M["p_mu.0.weight"], M["p_mu.0.bias"])), M["p_mu.2.weight"], M["p_mu.2.bias"])
    lv = torch.tanh(F.linear(F.relu(F.linear(x, M["p_logvar.0.weight"], M["p_logvar.0.bias"])),
                             M["p_logvar.2.weight"], M["p_logvar.2.bias"]))
    return mu, lv


def club_sample(M, x, y, perm):
    """CLUBSample.forward (mi_estimator.py:133-143) with the permutation passed in."""
    mu, lv = mlp_forward(M, x)
    positive = -((mu - y) ** 2) / lv.exp()
    negative = -((mu - y[perm]) ** 2) / lv.exp()
    return (positive.sum(dim=-1) - negative.sum(dim=-1)).mean() / 2.0


def l1out(M, x, y):
    """L1OutUB.forward (mi_estimator.py:170-191) including the [N,N,N] broadcast of diag_mask."""
    n = y.shape[0]
    mu, lv = mlp_forward(M, x)
    positive = (-((mu - y) ** 2) / 2.0 / lv.exp() - lv / 2.0).sum(dim=-1)
    all_probs = (-((y.unsqueeze(0) - mu.unsqueeze(1)) ** 2) / 2.0 / lv.unsqueeze(1).exp()
                 - lv.unsqueeze(1) / 2.0).sum(dim=-1)
    diag_mask = torch.ones([n], dtype=x.dtype).diag().unsqueeze(-1) * (-20.0)
    negative = logsumexp(all_probs + diag_mask, dim=0) - (torch.tensor(n) - 1.0).log().to(x.dtype)
    return (positive - negative).mean()


def learning_loss(M, x, y):
    """-loglikeli (mi_estimator.py:129-131)"""
    mu, lv = mlp_forward(M, x)
    return -((-((mu - y) ** 2) / lv.exp() - lv).sum(dim=1).mean(dim=0))


def anneal_weight(step, beta, loc=0, scale=1):
    """LogisticAnnealer.slope (trainer.py:32-34)"""
    return beta / (1 + math.exp(-(step - loc) / scale))


# ----------------------------------------------------------------------------- one training step


def clear_step(P, x, label, eps_c, eps_s, arch, hp, sim_fn="cosine", step=0, masks=None, bf16=False):
    """One CLEARVAETrainer step's losses and gradients (trainer.py:452-482), no optimizer update.  masks / bf16:
    encode / decode (test-side pinning of the device's ReLU activity and of its bf16 operand rounding)."""
    xhat, lp, z = vae_forward(P, x, eps_c, eps_s, arch, True, masks, bf16)
    rec, kl_c, kl_s = vae_loss(xhat, x, lp["mu_c"], lp["mu_s"], lp["logvar_c"], lp["logvar_s"])
    c = contrastive_loss(lp["mu_c"], lp["logvar_c"], label, sim_fn, hp["temperature"])
    s = contrastive_loss(lp["mu_s"], lp["logvar_s"], label, sim_fn, hp["temperature"], ps=hp["ps"])
    if not hp["ps"]:
        s = -s
    w = anneal_weight(step, hp["beta"], hp.get("loc", 0), hp.get("scale", 1))
    loss = rec + w * kl_c + w * kl_s + hp["alpha"] * c + hp["alpha"] * s
    params = {k: v for k, v in P.items() if isinstance(v, torch.Tensor) and v.requires_grad}
    grads = torch.autograd.grad(loss, list(params.values()), allow_unused=True)
    return {
        "xhat": xhat, "z": z, **lp, "rec": rec, "kl_c": kl_c, "kl_s": kl_s, "c_loss": c, "s_loss": s, "loss": loss,
        "grads": {k: g for k, g in zip(params, grads)},
    }


def mim_step(P, M, x, label, eps_c, eps_s, perm, arch, hp, kind="CLUBSample", sim_fn="cosine", step=0,
             masks=None, bf16=False):
    """The VAE half of one ClearMIMVAETrainer step (trainer.py:848-869): losses and VAE grads."""
    xhat, lp, z = vae_forward(P, x, eps_c, eps_s, arch, True, masks, bf16)
    rec, kl_c, kl_s = vae_loss(xhat, x, lp["mu_c"], lp["mu_s"], lp["logvar_c"], lp["logvar_s"])
    c = contrastive_loss(lp["mu_c"], lp["logvar_c"], label, sim_fn, hp["temperature"])
    d = z.shape[1] // 2
    mi = club_sample(M, z[:, :d], z[:, d:], perm) if kind == "CLUBSample" else l1out(M, z[:, :d], z[:, d:])
    w = anneal_weight(step, hp["beta"], hp.get("loc", 0), hp.get("scale", 1))
    loss = rec + w * kl_c + w * kl_s + hp["alpha"] * c + hp["lambda"] * mi
    params = {k: v for k, v in P.items() if isinstance(v, torch.Tensor) and v.requires_grad}
    grads = torch.autograd.grad(loss, list(params.values()), allow_unused=True)
    return {"xhat": xhat, "z": z, **lp, "rec": rec, "kl_c": kl_c, "kl_s": kl_s, "c_loss": c, "mi": mi,
            "loss": loss, "grads": {k: g for k, g in zip(params, grads)}}


# ----------------------------------------------------------------------------- CLEAR-TC


def disc_forward(D, z):
    """factor_cls(z) (trainer_utils.py:133-138): [n, 1] probabilities."""
    return torch.sigmoid(F.linear(F.relu(F.linear(z, D["0.weight"], D["0.bias"])), D["2.weight"], D["2.bias"]))


def factor_shuffling(z):
    """strategy "permute_1" (trainer.py:573-587): z_s rolled up by one row."""
    d = z.shape[1] // 2
    return torch.cat([z[:, :d], torch.cat([z[1:, d:], z[:1, d:]], dim=0)], dim=1)


def tc_mi_loss(D, z):
    """F.relu(torch.log(d_score / (1 - d_score))).mean() (trainer.py:664-665)."""
    d = disc_forward(D, z)
    return F.relu(torch.log(d / (1 - d))).mean()


def tc_step(P, D, x, label, eps_c, eps_s, arch, hp, sim_fn="cosine", step=0, masks=None):
    """The VAE half of one ClearTCVAETrainer step (trainer.py:654-677): losses and VAE grads (the
    discriminator's grads of this backward are discarded by factor_optimizer.zero_grad, :682)."""
    xhat, lp, z = vae_forward(P, x, eps_c, eps_s, arch, True, masks)
    rec, kl_c, kl_s = vae_loss(xhat, x, lp["mu_c"], lp["mu_s"], lp["logvar_c"], lp["logvar_s"])
    c = contrastive_loss(lp["mu_c"], lp["logvar_c"], label, sim_fn, hp["temperature"])
    mi = tc_mi_loss(D, z)
    w = anneal_weight(step, hp["beta"], hp.get("loc", 0), hp.get("scale", 1))
    loss = rec + w * kl_c + w * kl_s + hp["alpha"] * c + hp["lambda"] * mi
    params = {k: v for k, v in P.items() if isinstance(v, torch.Tensor) and v.requires_grad}
    grads = torch.autograd.grad(loss, list(params.values()), allow_unused=True)
    return {"xhat": xhat, "z": z, **lp, "rec": rec, "kl_c": kl_c, "kl_s": kl_s, "c_loss": c, "mi": mi,
            "loss": loss, "grads": {k: g for k, g in zip(params, grads)}}


def tc_factor_loss(D, z):
    """nn.BCELoss()(cat[factor_cls(z), factor_cls(factor_shuffling(z))], cat[1, 0]) (trainer.py:682-694);
    z is detached."""
    dj = disc_forward(D, z)
    dm = disc_forward(D, factor_shuffling(z))
    return F.binary_cross_entropy(torch.cat([dj, dm], dim=0), torch.cat([torch.ones_like(dj), torch.zeros_like(dm)]))


# ----------------------------------------------------------------------------- GVAE / ML-VAE


def group_evidence(mu_c, lv_c, label, mode):
    """accumulate_group_evidence (vae.py:159-190).  Groups are the sorted unique labels, members in
    ascending index.  As in the reference the group rows are held in torch.zeros(...) of the DEFAULT
    dtype (float32), so they are rounded to fp32 even in an fp64 run."""
    groups = torch.unique(label, sorted=True)
    mu_g = torch.zeros(len(groups), mu_c.shape[1])
    lv_g = torch.zeros(len(groups), lv_c.shape[1])
    members = {}
    for i, g in enumerate(groups):
        sel = label == g
        members[int(g)] = sel.nonzero().view(-1)
        if mode == "MLVAE":  # precision-weighted mean, log of the summed precisions
            lp = -lv_c[sel, :]
            lse = lp.logsumexp(dim=0)
            mu_g[i] = (mu_c[sel, :] * lp.exp()).sum(dim=0) * torch.exp(-lse)
            lv_g[i] = -lse
        elif mode == "GVAE":  # plain mean, log of the mean variance
            mu_g[i] = mu_c[sel, :].mean(dim=0)
            lv_g[i] = lv_c[sel, :].logsumexp(dim=0) - sel.sum().log()
        else:
            raise NotImplementedError("only support using MLVAE or GVAE")
    return mu_g, lv_g, members


def group_reparam(mu_g, lv_g, members, eps_sorted):
    """groupwise_reparam_each (vae.py:193-223) with the noise passed in: row r of eps_sorted belongs to
    the r-th sample in group order (the reference draws torch.randn(n_g, d) group after group)."""
    std = torch.exp(0.5 * lv_g)
    rows, idx, o = [], [], 0
    for i, (_, ix) in enumerate(members.items()):
        k = len(ix)
        rows.append(mu_g[i][None, :] + eps_sorted[o:o + k] * std[i][None, :])
        idx.append(ix)
        o += k
    z_sorted, idx = torch.cat(rows), torch.cat(idx)
    inverse = torch.zeros_like(idx)
    inverse[idx] = torch.arange(len(idx))
    return z_sorted[inverse]


def group_order_noise(label, eps_c):
    """The group-order rows of eps_c (sample-indexed) — the order the reference consumes noise in."""
    lab = torch.as_tensor(label)
    order = torch.cat([(lab == g).nonzero().view(-1) for g in torch.unique(lab, sorted=True)])
    return eps_c[order]


def group_step(P, x, label, eps_sorted, eps_s, arch, hp, mode, step=0, masks=None):
    """One HierarchicalVAETrainer step's losses and gradients (trainer.py:335-353), no optimizer update:
    the ELBO on the group rows for kl_c, rec and kl_s times B/m (_group_adjust, :322-324)."""
    mu_c, lv_c, mu_s, lv_s = encode(P, x, arch, True, masks)
    mu_g, lv_g, members = group_evidence(mu_c, lv_c, label, mode)
    z = torch.cat([group_reparam(mu_g, lv_g, members, eps_sorted), sample(mu_s, lv_s, eps_s)], dim=-1)
    xhat = decode(P, z, arch, True, masks)
    rec, kl_c, kl_s = vae_loss(xhat, x, mu_g, mu_s, lv_g, lv_s)
    B, m = x.shape[0], len(members)
    rec_a, kl_s_a = rec * B / m, kl_s * B / m
    w = anneal_weight(step, hp["beta"], hp.get("loc", 0), hp.get("scale", 1))
    loss = rec_a + w * kl_c + w * kl_s_a
    params = {k: v for k, v in P.items() if isinstance(v, torch.Tensor) and v.requires_grad}
    grads = torch.autograd.grad(loss, list(params.values()), allow_unused=True)
    return {"xhat": xhat, "z": z, "mu_c": mu_g, "logvar_c": lv_g, "mu_s": mu_s, "logvar_s": lv_s,
            "mu_c_sample": mu_c, "logvar_c_sample": lv_c, "rec": rec, "kl_c": kl_c, "kl_s": kl_s,
            "rec_adj": rec_a, "kl_s_adj": kl_s_a, "m": m, "loss": loss,
            "grads": {k: g for k, g in zip(params, grads)}}
