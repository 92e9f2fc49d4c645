"""Kernel-level parity of the implicit-GEMM conv / linear entry points against an fp64 host
computation of the same math (torch CPU ops on fp64 copies), at every CLEAR-VAE layer geometry,
with and without the fused BatchNorm prologue/epilogue transforms.  Tolerance: 1e-5 rel-L2 (fp32
MFMA accumulation over K <= 4096)."""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TOL = 1e-5


def rel(a, b):
    a = a.detach().double().cpu().reshape(-1)
    b = b.detach().double().cpu().reshape(-1)
    return float((a - b).norm() / (b.norm() + 1e-30))


# (n, transposed, c_in, h_in, c_out, h_out, k, s, p) : every conv of VAE (28x28) and VAE64 (64x64)
GEOMS = [
    (64, 0, 1, 28, 32, 14, 3, 2, 1), (64, 0, 32, 14, 64, 7, 3, 2, 1), (64, 0, 64, 7, 128, 4, 3, 2, 1),
    (64, 1, 128, 4, 64, 7, 3, 2, 1), (64, 1, 64, 7, 32, 14, 3, 2, 1), (64, 1, 32, 14, 1, 28, 3, 2, 1),
    (8, 0, 3, 64, 32, 32, 4, 2, 1), (8, 0, 32, 32, 64, 16, 4, 2, 1), (8, 0, 64, 16, 128, 8, 4, 2, 1),
    (8, 0, 128, 8, 256, 4, 4, 2, 1), (8, 0, 256, 4, 512, 2, 4, 2, 1),
    (8, 1, 512, 2, 256, 4, 4, 2, 1), (8, 1, 256, 4, 128, 8, 4, 2, 1), (8, 1, 128, 8, 64, 16, 4, 2, 1),
    (8, 1, 64, 16, 32, 32, 4, 2, 1), (8, 1, 32, 32, 3, 64, 4, 2, 1),
]


def _bn_state(C, count, rng, dev):
    """Random BN params + a consistent set of fp64 replica sums (stat, gstat) and host constants."""
    gamma = torch.tensor(rng.uniform(0.5, 1.5, C), dtype=torch.float32, device=dev)
    beta = torch.tensor(rng.uniform(-0.3, 0.3, C), dtype=torch.float32, device=dev)
    return gamma, beta


def _stats_of(t_nhwc, C):
    """fp64 replica-0 sums of an NHWC tensor (sum, sum of squares)."""
    v = t_nhwc.double().reshape(-1, C)
    from cvhip import _lib

    st = torch.zeros(_lib.stat_repl(C), 2, C, dtype=torch.float64, device=t_nhwc.device)
    st[0, 0] = v.sum(0)
    st[0, 1] = (v * v).sum(0)
    return st


def _cvbn(lib_mod, gamma, beta, stat, gstat, C, count, rm, rv):
    return lib_mod.cv_bn(gamma.data_ptr(), beta.data_ptr(), stat.data_ptr(),
                         gstat.data_ptr() if gstat is not None else None, rm.data_ptr(), rv.data_ptr(), C, count, 1, 1e-5)


def _host_bnrelu(y, gamma, beta, C):
    v = y.double().reshape(-1, C)
    m = v.mean(0)
    var = v.var(0, unbiased=False)
    out = torch.relu((v - m) / torch.sqrt(var + 1e-5) * gamma.double() + beta.double())
    return out.reshape(y.shape)


def _host_bnbwd(dz, y, gamma, C):
    v = y.double().reshape(-1, C)
    g = dz.double().reshape(-1, C)
    m = v.mean(0)
    var = v.var(0, unbiased=False)
    istd = 1.0 / torch.sqrt(var + 1e-5)
    xh = (v - m) * istd
    n = v.shape[0]
    dy = gamma.double() * istd * (g - g.sum(0) / n - xh * (g * xh).sum(0) / n)
    return dy.reshape(y.shape)


def _packed(lib_mod, W, tr):
    """(forward, backward-data) GEMM-native weight copies via cv_pack_conv_weights."""
    cs, cb, kh, kw = W.shape
    gat, sca = torch.empty_like(W), torch.empty_like(W)
    item = lib_mod.cv_conv_pack(W.data_ptr(), gat.data_ptr(), sca.data_ptr(), cs, cb, kh, kw)
    lib_mod.call("cv_pack_conv_weights", (lib_mod.cv_conv_pack * 1)(item), 1, lib_mod.stream_handle())
    torch.cuda.synchronize()
    # layout contract (include/clearvae.h): Wg[tap][cb][cs], Ws[tap][cs][cb]
    Wc = W.cpu()
    assert torch.equal(gat.cpu().view(kh, kw, cb, cs), Wc.permute(2, 3, 1, 0))
    assert torch.equal(sca.cpu().view(kh, kw, cs, cb), Wc.permute(2, 3, 0, 1))
    return (sca, gat) if tr else (gat, sca)


@pytest.fixture(params=["core", "generic"])
def gemm_kernel(request):
    """Run a test on the specialised GEMM core (default path) and on the generic kernel."""
    from cvhip import _lib

    prev = _lib.lib().cv_debug_force_generic_gemm(1 if request.param == "generic" else 0)
    yield request.param
    _lib.lib().cv_debug_force_generic_gemm(prev)


@pytest.mark.parametrize("geom", GEOMS, ids=lambda g: "T" * g[1] + f"{g[2]}x{g[3]}-{g[4]}x{g[5]}k{g[6]}")
@pytest.mark.parametrize("xf", ["none", "bn"])
def test_conv_fwd_bwd_wgrad(geom, xf, gemm_kernel):
    from cvhip import _lib

    n, tr, cin, hin, cout, hout, k, s, p = geom
    dev = torch.device("cuda")
    rng = np.random.default_rng(hash(geom) % 2**32)
    op = (hout - ((hin - 1) * s - 2 * p + k)) if tr else 0
    g = _lib.cv_conv(n, cin, hin, hin, cout, hout, hout, k, k, s, p, tr)
    wshape = (cin, cout, k, k) if tr else (cout, cin, k, k)
    W = torch.tensor(rng.uniform(-0.2, 0.2, wshape), dtype=torch.float32, device=dev)
    b = torch.tensor(rng.uniform(-0.2, 0.2, cout), dtype=torch.float32, device=dev)
    x = torch.tensor(rng.standard_normal((n, hin, hin, cin)), dtype=torch.float32, device=dev)  # NHWC
    dyo = torch.tensor(rng.standard_normal((n, hout, hout, cout)), dtype=torch.float32, device=dev)
    yo = torch.tensor(rng.standard_normal((n, hout, hout, cout)) * 2 + 0.5, dtype=torch.float32, device=dev)
    rm_i, rv_i = torch.zeros(cin, device=dev), torch.ones(cin, device=dev)
    rm_o, rv_o = torch.zeros(cout, device=dev), torch.ones(cout, device=dev)
    use_bn = xf == "bn" and cin % 1 == 0 and not (cin == 1 or cin == 3)
    s_ = _lib.stream_handle()
    Wf, Wb = _packed(_lib, W, tr)
    # ---------------- forward
    if use_bn:
        gi, bi = _bn_state(cin, n * hin * hin, rng, dev)
        st_i = _stats_of(x, cin)
        opnd = _lib.cv_operand(x.data_ptr(), None, _lib.XF_BNRELU, 0,
                               _cvbn(_lib, gi, bi, st_i, None, cin, n * hin * hin, rm_i, rv_i))
        xin_host = _host_bnrelu(x, gi, bi, cin)
    else:
        opnd = _lib.cv_operand(x.data_ptr(), None, _lib.XF_NONE, 0)
        xin_host = x.double()
    out = torch.empty(n, hout, hout, cout, dtype=torch.float32, device=dev)
    ep = _lib.cv_epilogue()
    ep.stat_mode, ep.stat_div = _lib.STAT_FWD, 1
    st_out = torch.zeros(_lib.stat_repl(cout), 2, cout, dtype=torch.float64, device=dev)
    ep.stat_out = st_out.data_ptr()
    _lib.call("cv_conv_forward", g, opnd, Wf.data_ptr(), b.data_ptr(), out.data_ptr(), ep, s_)
    xin_nchw = xin_host.permute(0, 3, 1, 2).cpu()
    Wd, bd = W.double().cpu(), b.double().cpu()
    if tr:
        ref = F.conv_transpose2d(xin_nchw, Wd, bd, stride=s, padding=p, output_padding=op)
    else:
        ref = F.conv2d(xin_nchw, Wd, bd, stride=s, padding=p)
    ref = ref.permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    assert rel(out, ref) < TOL, ("forward", rel(out, ref))
    ssum = st_out.sum(0).cpu()
    assert rel(ssum[0], ref.reshape(-1, cout).sum(0)) < 1e-6
    assert rel(ssum[1], (ref.reshape(-1, cout) ** 2).sum(0)) < 1e-6
    # ---------------- backward data (with BN-backward transform on dy when bn)
    if use_bn:  # (also the 1- / 3-channel image-side BN of the decoder output layer)
        go_, bo_ = _bn_state(cout, n * hout * hout, rng, dev)
        st_o = _stats_of(yo, cout)
        dz = dyo
        gst = torch.zeros(_lib.stat_repl(cout), 2, cout, dtype=torch.float64, device=dev)
        v = yo.double().reshape(-1, cout)
        xh = (v - v.mean(0)) / torch.sqrt(v.var(0, unbiased=False) + 1e-5)
        gst[0, 0] = dz.double().reshape(-1, cout).sum(0)
        gst[0, 1] = (dz.double().reshape(-1, cout) * xh).sum(0)
        gop = _lib.cv_operand(dz.data_ptr(), yo.data_ptr(), _lib.XF_BNBWD, 0,
                              _cvbn(_lib, go_, bo_, st_o, gst, cout, n * hout * hout, rm_o, rv_o))
        dy_host = _host_bnbwd(dz, yo, go_, cout)
    else:
        gop = _lib.cv_operand(dyo.data_ptr(), None, _lib.XF_NONE, 0)
        dy_host = dyo.double()
    gin = torch.empty(n, hin, hin, cin, dtype=torch.float32, device=dev)
    _lib.call("cv_conv_backward_data", g, gop, Wb.data_ptr(), gin.data_ptr(), _lib.cv_epilogue(), s_)
    dy_nchw = dy_host.permute(0, 3, 1, 2).cpu()
    if tr:
        gref = F.conv2d(dy_nchw, Wd, None, stride=s, padding=p)
    else:
        gref = torch.nn.grad.conv2d_input((n, cin, hin, hin), Wd, dy_nchw, stride=s, padding=p)
    gref = gref.permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    assert rel(gin, gref) < TOL, ("backward_data", rel(gin, gref))
    # ---------------- weight gradient (+ bias column when the layout allows): split-K partial tiles
    # through the workspace, then again with fp32 atomics (work = NULL)
    with_bias = (not tr) and (k * k * cin) % 4 == 0
    wb = _lib.lib().cv_conv_wgrad_workspace_bytes(g, 0)
    work = torch.empty(max(wb // 4, 1), dtype=torch.float32, device=dev)
    gw = torch.zeros(wshape, dtype=torch.float32, device=dev)
    gb = torch.zeros(cout, dtype=torch.float32, device=dev)
    _lib.call("cv_conv_backward_weight", g, opnd, gop, gw.data_ptr(), gb.data_ptr() if with_bias else None, 0,
              work.data_ptr(), wb, s_)
    gw_at = torch.full(wshape, 0.5, dtype=torch.float32, device=dev)  # accumulates onto existing values
    _lib.call("cv_conv_backward_weight", g, opnd, gop, gw_at.data_ptr(), None, 0, None, 0, s_)
    if tr:
        wref = torch.nn.grad.conv2d_weight(dy_nchw, (cin, cout, k, k), xin_nchw, stride=s, padding=p)
    else:
        wref = torch.nn.grad.conv2d_weight(xin_nchw, wshape, dy_nchw, stride=s, padding=p)
    torch.cuda.synchronize()
    assert rel(gw, wref) < TOL, ("backward_weight", rel(gw, wref))
    assert rel(gw_at - 0.5, wref) < TOL, ("backward_weight atomics", rel(gw_at - 0.5, wref))
    if with_bias:  # (a BN-backward dy sums to ~0 per channel: compare against the sum of |dy|)
        bref = dy_nchw.sum((0, 2, 3))
        err = float((gb.double().cpu() - bref).abs().max())
        assert err <= TOL * float(dy_nchw.abs().sum((0, 2, 3)).max()), ("bias grad", err)


@pytest.mark.parametrize("geom", [g for g in GEOMS if g[2] not in (1, 3)],
                         ids=lambda g: "T" * g[1] + f"{g[2]}x{g[3]}-{g[4]}x{g[5]}k{g[6]}")
def test_backward_data_stat_epilogue(geom, gemm_kernel, batch=16):
    """cv_conv_backward_data with CV_STAT_BWD: the stored tensor is dz = dx * [BN+ReLU active] and the
    fp64 sums are (sum dz, sum dz*xhat) of the BN layer that feeds this conv.  (batch: the pixel-major tests
    call it at batches that are multiples of the tile.)"""
    from cvhip import _lib

    n, tr, cin, hin, cout, hout, k, s, p = geom
    n = batch
    dev = torch.device("cuda")
    rng = np.random.default_rng(7 + hash(geom) % 1000)
    g = _lib.cv_conv(n, cin, hin, hin, cout, hout, hout, k, k, s, p, tr)
    wshape = (cin, cout, k, k) if tr else (cout, cin, k, k)
    W = torch.tensor(rng.uniform(-0.2, 0.2, wshape), dtype=torch.float32, device=dev)
    dyo = torch.tensor(rng.standard_normal((n, hout, hout, cout)), dtype=torch.float32, device=dev)
    yin = torch.tensor(rng.standard_normal((n, hin, hin, cin)) * 1.5 + 0.3, dtype=torch.float32, device=dev)
    gi, bi = _bn_state(cin, n * hin * hin, rng, dev)
    rm, rv = torch.zeros(cin, device=dev), torch.ones(cin, device=dev)
    st_i = _stats_of(yin, cin)
    gst = torch.zeros(_lib.stat_repl(cin), 2, cin, dtype=torch.float64, device=dev)
    ep = _lib.cv_epilogue()
    ep.stat_mode, ep.stat_div = _lib.STAT_BWD, 1
    ep.stat_out = gst.data_ptr()
    ep.ey = yin.data_ptr()
    ep.ebn = _cvbn(_lib, gi, bi, st_i, gst, cin, n * hin * hin, rm, rv)
    ep.erelu = 1
    gin = torch.empty(n, hin, hin, cin, dtype=torch.float32, device=dev)
    gop = _lib.cv_operand(dyo.data_ptr(), None, _lib.XF_NONE, 0)
    _, Wb = _packed(_lib, W, tr)
    _lib.call("cv_conv_backward_data", g, gop, Wb.data_ptr(), gin.data_ptr(), ep, _lib.stream_handle())
    Wd = W.double().cpu()
    dy_nchw = dyo.double().permute(0, 3, 1, 2).cpu()
    if tr:
        gref = F.conv2d(dy_nchw, Wd, None, stride=s, padding=p)
    else:
        gref = torch.nn.grad.conv2d_input((n, cin, hin, hin), Wd, dy_nchw, stride=s, padding=p)
    gref = gref.permute(0, 2, 3, 1).reshape(-1, cin)
    v = yin.double().cpu().reshape(-1, cin)
    m, var = v.mean(0), v.var(0, unbiased=False)
    xh = (v - m) / torch.sqrt(var + 1e-5)
    act = xh * gi.double().cpu() + bi.double().cpu()
    dz = gref * (act > 0)
    torch.cuda.synchronize()
    assert rel(gin.reshape(-1, cin), dz) < TOL, rel(gin.reshape(-1, cin), dz)
    sums = gst.sum(0).cpu()
    assert rel(sums[0], dz.sum(0)) < 1e-5
    assert rel(sums[1], (dz * xh).sum(0)) < 1e-5
