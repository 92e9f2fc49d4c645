"""cv_conv_backward_deferred on the image-side ConvTranspose2d (vae.py:43 / :153): the one-launch
edge_bwd_kernel against the two separate calls it replaces (cv_conv_backward_data + cv_conv_backward_weight_deferred)
on the same operands.  The fused kernel stages and contracts exactly as edge_gather_kernel / edge_wgrad_kernel, so
the data gradient and the weight-gradient partial tiles must be bit-identical; the BN backward sums are fp64
atomics (arrival order varies) and are held at 1e-12.  The reduced weight gradient (cv_step_reduce over the
deferred partials) is also checked against an fp64 torch conv_transpose2d weight gradient at 1e-5."""

import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GEOS = [  # n, c_small (=32), h_small, c_big, h_big, k, s, p, output_padding  (MNIST convT3, VAE64 convT5)
    (64, 32, 14, 1, 28, 3, 2, 1, 1),
    (16, 32, 32, 3, 64, 4, 2, 1, 0),
    (5, 32, 14, 1, 28, 3, 2, 1, 1),
]


def _bn(lib, dev, C, count, g, with_grad):
    R = lib.stat_repl(C)
    mean = torch.tensor(g.uniform(-0.2, 0.2, C))
    var = torch.tensor(g.uniform(0.5, 1.5, C))
    st = torch.zeros(R, 2, C, dtype=torch.float64)
    st[0, 0] = mean * count
    st[0, 1] = (var + mean * mean) * count
    gs = torch.zeros(R, 2, C, dtype=torch.float64)
    if with_grad:
        gs[0, 0] = torch.tensor(g.uniform(-1, 1, C)) * count * 0.01
        gs[0, 1] = torch.tensor(g.uniform(-1, 1, C)) * count * 0.01
    t = dict(stat=st.to(dev), gstat=gs.to(dev),
             gamma=torch.tensor(g.uniform(0.5, 1.5, C), dtype=torch.float32, device=dev),
             beta=torch.tensor(g.uniform(-0.3, 0.3, C), dtype=torch.float32, device=dev),
             rm=torch.zeros(C, device=dev), rv=torch.ones(C, device=dev))
    s = lib.cv_bn(t["gamma"].data_ptr(), t["beta"].data_ptr(), t["stat"].data_ptr(), t["gstat"].data_ptr(),
                  t["rm"].data_ptr(), t["rv"].data_ptr(), C, count, 1, 1e-5, None, None, None)
    return s, t


@pytest.mark.parametrize("geo", GEOS, ids=lambda v: "x".join(map(str, v)))
def test_edge_bwd_matches_separate_calls(geo):
    from cvhip import _lib

    n, cs, hs, cb, hb, k, s, p, op = geo
    dev = torch.device("cuda")
    lib = _lib
    g = np.random.default_rng(n * hs + cb)
    conv = _lib.cv_conv(n, cs, hs, hs, cb, hb, hb, k, k, s, p, 1, 0)
    bnb, tb = _bn(lib, dev, cb, n * hb * hb, g, True)     # the image-side BatchNorm (gout's BN backward)
    bns, ts = _bn(lib, dev, cs, n * hs * hs, g, False)    # the small side's BatchNorm (epilogue + X transform)
    dy = torch.tensor(g.standard_normal((n, hb, hb, cb)), dtype=torch.float32, device=dev)
    yb = torch.tensor(g.standard_normal((n, hb, hb, cb)), dtype=torch.float32, device=dev)
    ys = torch.tensor(g.standard_normal((n, hs, hs, cs)), dtype=torch.float32, device=dev)
    W = torch.tensor(g.uniform(-0.2, 0.2, (cs, cb, k, k)), dtype=torch.float32, device=dev)  # ConvT [Cin][Cout][kh][kw]
    wg = W.permute(2, 3, 1, 0).contiguous()  # gather packing [tap][cb][cs]
    gout = _lib.cv_operand(dy.data_ptr(), yb.data_ptr(), _lib.XF_BNBWD, 0, bnb)
    xin = _lib.cv_operand(ys.data_ptr(), None, _lib.XF_BNRELU, 0, bns)
    wb = int(lib.lib().cv_conv_wgrad_workspace_bytes(ctypes.byref(conv), 0))
    L = lib.lib()
    st = lib.stream_handle()
    out = {}
    for fused in (True, False):
        gst = torch.zeros_like(ts["gstat"])
        ep = _lib.cv_epilogue()
        ep.stat_mode = _lib.STAT_BWD
        ep.stat_out = gst.data_ptr()
        ep.stat_div = 1
        ep.ey = ys.data_ptr()
        ep.ebn = bns
        ep.erelu = 1
        gin = torch.full((n, hs, hs, cs), 7.0, device=dev)
        gw = torch.zeros(cs, cb, k, k, device=dev)
        work = torch.full((wb // 4 + 4,), 3.0, device=dev)
        d = _lib.cv_wgrad_defer()
        if fused:
            lib.call("cv_conv_backward_deferred", ctypes.byref(conv), ctypes.byref(gout), wg.data_ptr(), gin.data_ptr(),
                     ctypes.byref(ep), ctypes.byref(xin), gw.data_ptr(), None, work.data_ptr(), work.numel() * 4,
                     ctypes.byref(d), st)
        else:
            lib.call("cv_conv_backward_data", ctypes.byref(conv), ctypes.byref(gout), wg.data_ptr(), gin.data_ptr(),
                     ctypes.byref(ep), st)
            lib.call("cv_conv_backward_weight_deferred", ctypes.byref(conv), ctypes.byref(xin), ctypes.byref(gout),
                     gw.data_ptr(), None, work.data_ptr(), work.numel() * 4, ctypes.byref(d), st)
        torch.cuda.synchronize()
        nparts = d.split * d.M * d.ntot
        assert d.split > 0 and d.part == work.data_ptr()
        # reduce the deferred partials (cv_step_reduce with no BN layers)
        arr = (_lib.cv_wgrad_defer * 1)(d)
        lib.call("cv_step_reduce", arr, 1, None, 0, None, None, 0, ctypes.c_float(0.1), None, st)
        torch.cuda.synchronize()
        out[fused] = (gin.clone(), work[:nparts].clone(), gst.clone(), gw.clone())
    a, b = out[True], out[False]
    assert torch.equal(a[0], b[0]), "data gradient differs from edge_gather"
    assert torch.equal(a[1], b[1]), "weight-gradient partials differ from edge_wgrad"
    assert float((a[2] - b[2]).abs().max()) <= 1e-12 * max(1.0, float(b[2].abs().max()))
    assert torch.equal(a[3], b[3])
    # the reduced weight gradient against fp64 torch: dW = conv_transpose2d weight grad of relu(bn(ys)), bn_bwd(dy)
    def bn_consts(t, C, count):
        s0 = t["stat"][:, 0].sum(0).cpu()
        s1 = t["stat"][:, 1].sum(0).cpu()
        mean = s0 / count
        var = (s1 / count - mean * mean).clamp_min(0)
        return mean, 1.0 / torch.sqrt(var + 1e-5)

    mu_s, is_s = bn_consts(ts, cs, n * hs * hs)
    xs = torch.relu((ys.double().cpu() - mu_s) * is_s * ts["gamma"].double().cpu() + ts["beta"].double().cpu())
    mu_b, is_b = bn_consts(tb, cb, n * hb * hb)
    cnt = n * hb * hb
    c1 = tb["gstat"][:, 0].sum(0).cpu() / cnt
    c2 = tb["gstat"][:, 1].sum(0).cpu() / cnt
    dyt = tb["gamma"].double().cpu() * is_b * (dy.double().cpu() - c1 - (yb.double().cpu() - mu_b) * is_b * c2)
    xs_ = xs.permute(0, 3, 1, 2).requires_grad_(False)
    w_ = W.double().cpu().requires_grad_(True)
    yt = torch.nn.functional.conv_transpose2d(xs_, w_, stride=s, padding=p, output_padding=op)
    yt.backward(dyt.permute(0, 3, 1, 2))
    ref = w_.grad
    rel = float((a[3].double().cpu() - ref).norm() / ref.norm())
    assert rel < 1e-5, rel
