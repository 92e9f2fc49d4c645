"""The fused decoder-input block (cv_decoder_input_forward / _backward, cv_declinear.hip) against fp64 torch
restatements of the reference's VAE.sample -> decoder Linear -> BatchNorm1d -> ReLU
(code/src/models/vae.py:56-60, :33-35) and its backward, at the MNIST (z=16, Unflatten(128, 4, 4)) and VAE64
(z=64, Unflatten(512, 2, 2)) shapes and a ragged batch.

Tolerances: z is bit-identical to cv_reparam_forward (same Philox draw, same arithmetic); h, ah, the BN1d
sums, d(h) and the weight gradient within 1e-5 relative L2 of fp64 (fp32 contractions of length 2d and n).
The ReLU mask of the reference is taken from the kernel's own ah > 0, so elements within fp32 rounding of the
ReLU edge cannot flip between the two evaluations."""

import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [  # n, d (latent half-width), Cu, Hu*Wu
    (512, 8, 128, 16),
    (256, 32, 512, 4),
    (37, 8, 128, 16),
]


def _rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _bn_struct(gamma, beta, stat, gstat, rmean, rvar, C, count, train):
    from cvhip import _lib

    return _lib.cv_bn(gamma.data_ptr(), beta.data_ptr(), stat.data_ptr(), gstat.data_ptr(), rmean.data_ptr(),
                      rvar.data_ptr(), C, count, int(train), 1e-5, None, None, None)


def _storage(t, pix, ch):
    """[n][F] PyTorch feature order (c * pix + p) -> Unflatten/NHWC storage order (p * ch + c)."""
    n = t.shape[0]
    return t.view(n, ch, pix).permute(0, 2, 1).reshape(n, pix * ch)


@pytest.mark.parametrize("n,d,ch,pix", CASES)
def test_decoder_input_forward_backward(n, d, ch, pix):
    from cvhip import _lib

    dev = torch.device("cuda")
    L = _lib.lib()
    F, K = ch * pix, 2 * d
    assert L.cv_decoder_input_supported(n, d, F) == 1
    g = np.random.default_rng(n + d)
    heads = torch.tensor(g.standard_normal((n, 4 * d)) * 0.5, dtype=torch.float32, device=dev)
    W = torch.tensor(g.uniform(-0.3, 0.3, (F, K)), dtype=torch.float32, device=dev)
    b = torch.tensor(g.uniform(-0.2, 0.2, F), dtype=torch.float32, device=dev)
    gamma = torch.tensor(g.uniform(0.5, 1.5, F), dtype=torch.float32, device=dev)
    beta = torch.tensor(g.uniform(-0.3, 0.3, F), dtype=torch.float32, device=dev)
    rmean = torch.zeros(F, device=dev)
    rvar = torch.ones(F, device=dev)
    R = _lib.stat_repl(F)
    stat = torch.zeros(R, 2, F, dtype=torch.float64, device=dev)
    gstat = torch.zeros(R, 2, F, dtype=torch.float64, device=dev)
    lin = _lib.cv_linear(n, K, F, 1, 0, pix, ch, 0)
    bn = _bn_struct(gamma, beta, stat, gstat, rmean, rvar, F, n, True)
    seed = 1234
    off = torch.tensor([5, 0], dtype=torch.int64, device=dev)
    off_ref = torch.tensor([5, 0], dtype=torch.int64, device=dev)
    z = torch.empty(n, K, device=dev)
    z_ref = torch.empty(n, K, device=dev)
    h = torch.empty(n, F, device=dev)
    ah = torch.empty(n, F, device=dev)
    s = _lib.stream_handle()
    _lib.call("cv_reparam_forward", heads.data_ptr(), n, d, None, ctypes.c_uint64(seed), off_ref.data_ptr(),
              z_ref.data_ptr(), None, s)
    _lib.call("cv_decoder_input_forward", ctypes.byref(lin), heads.data_ptr(), None, ctypes.c_uint64(seed),
              off.data_ptr(), z.data_ptr(), W.data_ptr(), b.data_ptr(), ctypes.byref(bn), stat.data_ptr(),
              h.data_ptr(), ah.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(z, z_ref), "z differs from cv_reparam_forward's draw"
    assert off.tolist() == [6, 0] and off_ref.tolist() == [6, 0]
    # fp64 restatement (PyTorch feature order), then to storage order
    zd = z.double()
    hd = zd @ W.double().T + b.double()
    mean = hd.mean(0)
    var = hd.var(0, unbiased=False)
    xhat = (hd - mean) / torch.sqrt(var + 1e-5)
    ad = torch.relu(xhat * gamma.double() + beta.double())
    assert _rel(h, _storage(hd, pix, ch)) < 1e-5
    assert _rel(ah, _storage(ad, pix, ch)) < 1e-5
    assert _rel(stat[0, 0], hd.sum(0)) < 1e-6 and _rel(stat[0, 1], (hd * hd).sum(0)) < 1e-6
    assert float(stat[1:].abs().max()) == 0.0

    # backward: ga = d(ReLU output) in storage order
    ga_pt = torch.tensor(g.standard_normal((n, F)), dtype=torch.float64, device=dev)
    ga = _storage(ga_pt, pix, ch).float().contiguous()
    gw = torch.zeros(F, K, device=dev)
    dzo = torch.zeros(n, K, device=dev)
    _lib.call("cv_decoder_input_backward", ctypes.byref(lin), ga.data_ptr(), h.data_ptr(), ctypes.byref(bn),
              gstat.data_ptr(), z.data_ptr(), gw.data_ptr(), W.data_ptr(), dzo.data_ptr(), s)
    torch.cuda.synchronize()
    # the kernel's own ReLU decisions: the backward re-derives the forward's constants from the same sums, so
    # its mask is the forward's ah > 0
    istd32 = 1.0 / torch.sqrt(var + 1e-5)
    mask = (ah > 0).view(n, pix, ch).permute(0, 2, 1).reshape(n, F)
    dz = ga_pt * mask
    c1 = dz.mean(0)
    c2 = (dz * xhat).mean(0)
    dh = gamma.double() * istd32 * (dz - c1 - xhat * c2)
    assert _rel(gstat[0, 0], dz.sum(0)) < 1e-6 and _rel(gstat[0, 1], (dz * xhat).sum(0)) < 1e-5
    assert _rel(ga, _storage(dh, pix, ch)) < 1e-5
    assert _rel(gw, dh.T @ zd) < 1e-5
    assert _rel(dzo, dh @ W.double()) < 1e-5


def test_decoder_input_eval_and_given_z():
    """Eval mode (running statistics) with z given (the generate / module path)."""
    from cvhip import _lib

    dev = torch.device("cuda")
    n, d, ch, pix = 64, 8, 128, 16
    F, K = ch * pix, 2 * d
    g = np.random.default_rng(7)
    z = torch.tensor(g.standard_normal((n, K)), dtype=torch.float32, device=dev)
    W = torch.tensor(g.uniform(-0.3, 0.3, (F, K)), dtype=torch.float32, device=dev)
    b = torch.tensor(g.uniform(-0.2, 0.2, F), dtype=torch.float32, device=dev)
    gamma = torch.tensor(g.uniform(0.5, 1.5, F), dtype=torch.float32, device=dev)
    beta = torch.tensor(g.uniform(-0.3, 0.3, F), dtype=torch.float32, device=dev)
    rmean = torch.tensor(g.uniform(-0.5, 0.5, F), dtype=torch.float32, device=dev)
    rvar = torch.tensor(g.uniform(0.5, 2.0, F), dtype=torch.float32, device=dev)
    stat = torch.zeros(_lib.stat_repl(F), 2, F, dtype=torch.float64, device=dev)
    lin = _lib.cv_linear(n, K, F, 1, 0, pix, ch, 0)
    bn = _bn_struct(gamma, beta, stat, stat, rmean, rvar, F, n, False)
    h = torch.empty(n, F, device=dev)
    ah = torch.empty(n, F, device=dev)
    z0 = z.clone()
    _lib.call("cv_decoder_input_forward", ctypes.byref(lin), None, None, ctypes.c_uint64(0), None, z.data_ptr(),
              W.data_ptr(), b.data_ptr(), ctypes.byref(bn), None, h.data_ptr(), ah.data_ptr(), _lib.stream_handle())
    torch.cuda.synchronize()
    assert torch.equal(z, z0)
    hd = z.double() @ W.double().T + b.double()
    ad = torch.relu((hd - rmean.double()) / torch.sqrt(rvar.double() + 1e-5) * gamma.double() + beta.double())
    assert _rel(h, _storage(hd, pix, ch)) < 1e-5
    assert _rel(ah, _storage(ad, pix, ch)) < 1e-5
    assert float(stat.abs().max()) == 0.0


HEADS = [  # n, C, pix (Hh*Wh), J = 4d
    (512, 128, 16, 32),
    (256, 512, 4, 128),
    (37, 128, 16, 32),
]


@pytest.mark.parametrize("n,C,pix,J", HEADS)
@pytest.mark.parametrize("finalise", [False, True])
def test_heads_backward(n, C, pix, J, finalise):
    """cv_heads_backward (the heads' nn.Linear backward, vae.py:25-30, with the last encoder block's BN + ReLU
    backward mask and sums) against fp64; with a ticket, the last workgroup's finalised BN backward constants."""
    from cvhip import _lib

    dev = torch.device("cuda")
    F = C * pix
    assert _lib.lib().cv_heads_backward_supported(n, F, C, J) == 1
    g = np.random.default_rng(n + J)
    dheads = torch.tensor(g.standard_normal((n, J)), dtype=torch.float32, device=dev)
    W = torch.tensor(g.uniform(-0.05, 0.05, (J, F)), dtype=torch.float32, device=dev)
    y = torch.tensor(g.standard_normal((n, F)) + 0.3, dtype=torch.float32, device=dev)  # storage order
    gamma = torch.tensor(g.uniform(0.5, 1.5, C), dtype=torch.float32, device=dev)
    beta = torch.tensor(g.uniform(-0.3, 0.3, C), dtype=torch.float32, device=dev)
    R = _lib.stat_repl(C)
    yc = y.double().view(n * pix, C)  # (n, pixel) x channel
    stat = torch.zeros(R, 2, C, dtype=torch.float64, device=dev)
    stat[0, 0] = yc.sum(0)
    stat[0, 1] = (yc * yc).sum(0)
    gstat = torch.zeros(R, 2, C, dtype=torch.float64, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    cbwd = torch.zeros(5 * C, device=dev)
    ticket = torch.zeros(_lib.TICKET_WORDS, dtype=torch.int32, device=dev)
    bn = _lib.cv_bn(gamma.data_ptr(), beta.data_ptr(), stat.data_ptr(), gstat.data_ptr(), rm.data_ptr(),
                    rv.data_ptr(), C, n * pix, 1, 1e-5, None, cbwd.data_ptr() if finalise else None,
                    ticket.data_ptr() if finalise else None)
    lin = _lib.cv_linear(n, F, J, pix, C, 1, 0, 0)
    gin = torch.empty(n, F, device=dev)
    gw = torch.zeros(J, F, device=dev)
    gb = torch.zeros(J, device=dev)
    _lib.call("cv_heads_backward", ctypes.byref(lin), dheads.data_ptr(), W.data_ptr(), y.data_ptr(),
              ctypes.byref(bn), gin.data_ptr(), gstat.data_ptr(), gw.data_ptr(), gb.data_ptr(), _lib.stream_handle())
    torch.cuda.synchronize()
    mean = yc.mean(0)
    var = yc.var(0, unbiased=False)
    istd = 1.0 / torch.sqrt(var + 1e-5)
    xh = ((yc - mean) * istd).view(n, F)  # storage order
    o = xh * gamma.double().repeat(pix) + beta.double().repeat(pix)
    mask = gin != 0  # the kernel's own ReLU decisions (a masked element is exactly 0)
    edge = o.abs() < 1e-5
    assert bool(((o > 0) == mask)[~edge].all()), "ReLU mask differs away from the edge"
    gflat_pt = dheads.double() @ W.double()  # PyTorch feature order c*pix + p
    gflat = gflat_pt.view(n, C, pix).permute(0, 2, 1).reshape(n, F)
    dz = gflat * mask
    assert _rel(gin, dz) < 1e-5
    a_pt = torch.relu(o).view(n, pix, C).permute(0, 2, 1).reshape(n, F)
    assert _rel(gw, dheads.double().T @ a_pt) < 1e-5
    assert _rel(gb, dheads.double().sum(0)) < 1e-5
    dzc = dz.view(n * pix, C)
    s1 = gstat[:, 0].sum(0)
    s2 = gstat[:, 1].sum(0)
    assert _rel(s1, dzc.sum(0)) < 1e-5 and _rel(s2, (dzc * xh.view(n * pix, C)).sum(0)) < 1e-5
    if finalise:
        cnt = n * pix
        ref = torch.cat([gamma.double() * istd, dzc.sum(0) / cnt, mean, istd,
                         (dzc * xh.view(n * pix, C)).sum(0) / cnt])
        assert _rel(cbwd, ref) < 1e-5
        nblk = F // 16  # two-level arrival count (include/clearvae.h cv_bn.ticket): groups done
        gsz = (nblk + 63) // 64
        assert int(ticket[1]) == (nblk + gsz - 1) // gsz
    else:
        assert float(cbwd.abs().max()) == 0.0


def _chain_torch(dheads, heads, z, dz, d):
    """dheads + the decoder chain term of cv_latent_combine (vae.py:56-60 through z = mu + eps exp(lv / 2)), in
    the kernel's fp32 operation order."""
    full = dheads.clone()
    for b in range(4):
        zi = slice((b >> 1) * d, (b >> 1) * d + d)
        cols = slice(b * d, (b + 1) * d)
        if b % 2 == 0:
            full[:, cols] = dheads[:, cols] + dz[:, zi]
        else:
            full[:, cols] = dheads[:, cols] + dz[:, zi] * (z[:, zi] - heads[:, (b - 1) * d:b * d]) * 0.5
    return full


@pytest.mark.parametrize("n,C,pix,J", HEADS)
def test_heads_backward_chain(n, C, pix, J):
    """cv_heads_backward_chain (the decoder chain term added while dheads is staged, engine LATENT_CHAIN) is
    cv_heads_backward of dheads + that term: bit-identical d(input) (the weight / bias gradients to 1e-6 and the BN
    backward sums, fp64 atomics of several workgroups, to 1e-12: summation order only), dheads left as it was,
    losses[0] = the rec replicas' sum."""
    from cvhip import _lib

    dev = torch.device("cuda")
    F, d = C * pix, J // 4
    g = np.random.default_rng(7 * n + J)
    t = lambda *sh: torch.tensor(g.standard_normal(sh), dtype=torch.float32, device=dev)
    dheads, heads, z, dz = t(n, J), t(n, J), t(n, 2 * d), t(n, 2 * d)
    W = torch.tensor(g.uniform(-0.05, 0.05, (J, F)), dtype=torch.float32, device=dev)
    y = t(n, F) + 0.3
    gamma = torch.tensor(g.uniform(0.5, 1.5, C), dtype=torch.float32, device=dev)
    beta = torch.tensor(g.uniform(-0.3, 0.3, C), dtype=torch.float32, device=dev)
    R = _lib.stat_repl(C)
    yc = y.double().view(n * pix, C)
    stat = torch.zeros(R, 2, C, dtype=torch.float64, device=dev)
    stat[0, 0] = yc.sum(0)
    stat[0, 1] = (yc * yc).sum(0)
    rec = torch.tensor(g.uniform(0, 1, _lib.REC_REPL), dtype=torch.float64, device=dev)
    losses = torch.zeros(24, device=dev)
    lin = _lib.cv_linear(n, F, J, pix, C, 1, 0, 0)
    outs = []
    for chained in (True, False):
        gstat = torch.zeros(R, 2, C, dtype=torch.float64, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        bn = _lib.cv_bn(gamma.data_ptr(), beta.data_ptr(), stat.data_ptr(), gstat.data_ptr(), rm.data_ptr(),
                        rv.data_ptr(), C, n * pix, 1, 1e-5, None, None, None)
        gin = torch.empty(n, F, device=dev)
        gw = torch.zeros(J, F, device=dev)
        gb = torch.zeros(J, device=dev)
        before = dheads.clone()
        if chained:
            ch = _lib.cv_latent_chain(heads.data_ptr(), z.data_ptr(), dz.data_ptr(), d, rec.data_ptr(),
                                      losses.data_ptr())
            _lib.call("cv_heads_backward_chain", ctypes.byref(lin), dheads.data_ptr(), ctypes.byref(ch), W.data_ptr(),
                      y.data_ptr(), ctypes.byref(bn), gin.data_ptr(), gstat.data_ptr(), gw.data_ptr(), gb.data_ptr(),
                      _lib.stream_handle())
        else:
            full = _chain_torch(dheads, heads, z, dz, d)
            _lib.call("cv_heads_backward", ctypes.byref(lin), full.data_ptr(), W.data_ptr(), y.data_ptr(),
                      ctypes.byref(bn), gin.data_ptr(), gstat.data_ptr(), gw.data_ptr(), gb.data_ptr(),
                      _lib.stream_handle())
        torch.cuda.synchronize()
        assert torch.equal(dheads, before)
        outs.append((gin.cpu(), gw.cpu(), gb.cpu(), gstat.cpu()))
    assert torch.equal(outs[0][0].view(torch.int32), outs[1][0].view(torch.int32)), (outs[0][0] - outs[1][0]).abs().max()
    # (gw / gb: the plain launch splits the rows of a large batch over two workgroups whose sums meet in atomics, the
    # chained one does not: the same sums in another order)
    for a, b, name in zip(outs[0][1:3], outs[1][1:3], ("gw", "gb")):
        assert _rel(a, b) < 1e-6, (name, _rel(a, b))
    assert _rel(outs[0][3], outs[1][3]) < 1e-12
    r = 0.0
    for v in rec.cpu().tolist():  # (the kernel's order)
        r += v
    assert float(losses[0]) == float(np.float32(r))


HEADS_FWD = [  # n, C, (Hh, Wh), d
    (512, 128, (4, 4), 8),
    (256, 512, (2, 2), 32),
    (37, 128, (4, 4), 8),
]


@pytest.mark.parametrize("n,C,hw,d", HEADS_FWD)
@pytest.mark.parametrize("finalised", [False, True])
def test_heads_forward_reparam(n, C, hw, d, finalised):
    """cv_heads_forward (vae.py:25-30 heads on ReLU(BN(y)), then VAE.sample vae.py:56-60) against fp64, with the
    weight packed by cv_pack_conv_weights; z bit-identical to cv_reparam_forward on the kernel's heads."""
    from cvhip import _lib

    dev = torch.device("cuda")
    Hh, Wh = hw
    pix, F, J = Hh * Wh, C * Hh * Wh, 4 * d
    assert _lib.lib().cv_heads_forward_supported(n, F, C, d) == 1
    g = np.random.default_rng(n + d + C)
    y = torch.tensor(g.standard_normal((n, F)) + 0.2, dtype=torch.float32, device=dev)  # storage order
    W = torch.tensor(g.uniform(-0.05, 0.05, (J, F)), dtype=torch.float32, device=dev)
    b = torch.tensor(g.uniform(-0.1, 0.1, J), dtype=torch.float32, device=dev)
    gamma = torch.tensor(g.uniform(0.5, 1.5, C), dtype=torch.float32, device=dev)
    beta = torch.tensor(g.uniform(-0.3, 0.3, C), dtype=torch.float32, device=dev)
    yc = y.double().view(n * pix, C)
    mean, var = yc.mean(0), yc.var(0, unbiased=False)
    istd = 1.0 / torch.sqrt(var + 1e-5)
    R = _lib.stat_repl(C)
    stat = torch.zeros(R, 2, C, dtype=torch.float64, device=dev)
    stat[0, 0] = yc.sum(0)
    stat[0, 1] = (yc * yc).sum(0)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    cfwd = torch.cat([(gamma.double() * istd), mean, beta.double(), istd]).float().to(dev)
    ticket = torch.zeros(_lib.TICKET_WORDS, dtype=torch.int32, device=dev)
    ticket[0] = 1
    bn = _lib.cv_bn(gamma.data_ptr(), beta.data_ptr(), stat.data_ptr(), stat.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                    C, n * pix, 1, 1e-5, None if not finalised else None, None, None)
    if finalised:
        bn.cfwd = cfwd.data_ptr()
        bn.ticket = ticket.data_ptr()
    wp = torch.empty(F * J, device=dev)
    item = (_lib.cv_conv_pack * 1)(_lib.cv_conv_pack(W.data_ptr(), wp.data_ptr(), None, J, C, Hh, Wh))
    s = _lib.stream_handle()
    _lib.call("cv_pack_conv_weights", item, 1, s)
    lin = _lib.cv_linear(n, F, J, pix, C, 1, 0, 0)
    heads = torch.empty(n, J, device=dev)
    z = torch.empty(n, 2 * d, device=dev)
    off = torch.tensor([3, 0], dtype=torch.int64, device=dev)
    _lib.call("cv_heads_forward", ctypes.byref(lin), y.data_ptr(), ctypes.byref(bn), wp.data_ptr(), b.data_ptr(),
              heads.data_ptr(), None, ctypes.c_uint64(99), off.data_ptr(), z.data_ptr(), s)
    z_ref = torch.empty(n, 2 * d, device=dev)
    off_ref = torch.tensor([3, 0], dtype=torch.int64, device=dev)
    _lib.call("cv_reparam_forward", heads.data_ptr(), n, d, None, ctypes.c_uint64(99), off_ref.data_ptr(),
              z_ref.data_ptr(), None, s)
    torch.cuda.synchronize()
    a = torch.relu(((yc - mean) * istd * gamma.double() + beta.double())).view(n, pix, C).permute(0, 2, 1)
    ref = a.reshape(n, F) @ W.double().T + b.double()
    assert _rel(heads, ref) < 1e-5
    assert torch.equal(z, z_ref), "z differs from cv_reparam_forward on the same heads"
    assert off.tolist() == [4, 0]
