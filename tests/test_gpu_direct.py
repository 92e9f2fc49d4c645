"""The class-fused direct SCATTER kernel (cv_direct.hip, reached through cv_conv_forward_kpack /
cv_conv_backward_data_kpack): Conv2d backward-data and ConvTranspose2d forward at every stride-2 geometry of VAE
and VAE64 it serves (vae.py:15-46, 113-156), with and without the fused BatchNorm transforms and statistics
epilogues, at small, ragged and the bench's full batches.

Each case is checked three ways:
  * the direct kernel really ran (cv_debug_direct_count), or — for the geometries it does not serve (VAE64's
    256 / 512-channel layers) — the kpack call fell back to the GEMM core;
  * against an fp64 torch evaluation of the same math at the kernel bar 1e-5 (tests/test_gpu_conv_kernels.py),
    including the epilogue's fp64 batch sums;
  * against the per-class GEMM core on the same operands (cv_conv_forward / cv_conv_backward_data): the same
    contraction summed in another order, so within 2e-6 relative."""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from test_gpu_conv_kernels import TOL, _bn_state, _cvbn, _host_bnbwd, _host_bnrelu, _packed, _stats_of, rel

pytestmark = pytest.mark.gpu

# (n, transposed, c_in, h_in, c_out, h_out, k, s, p): the stride-2 layers whose SCATTER half the kernel serves
# (Conv2d: backward-data; ConvTranspose2d: forward)
SERVED = [
    (16, 0, 32, 14, 64, 7, 3, 2, 1), (16, 0, 64, 7, 128, 4, 3, 2, 1),        # MNIST conv2 / conv3
    (16, 1, 128, 4, 64, 7, 3, 2, 1), (16, 1, 64, 7, 32, 14, 3, 2, 1),        # MNIST convT1 / convT2
    (8, 0, 32, 32, 64, 16, 4, 2, 1), (8, 0, 64, 16, 128, 8, 4, 2, 1),        # VAE64 conv2 / conv3
    (8, 1, 128, 8, 64, 16, 4, 2, 1), (8, 1, 64, 16, 32, 32, 4, 2, 1),        # VAE64 convT3 / convT4
    (5, 0, 32, 14, 64, 7, 3, 2, 1), (3, 1, 128, 8, 64, 16, 4, 2, 1),         # ragged batches
    (512, 0, 32, 14, 64, 7, 3, 2, 1), (512, 1, 64, 7, 32, 14, 3, 2, 1),      # the MNIST bench batch
    (256, 0, 32, 32, 64, 16, 4, 2, 1), (128, 1, 128, 8, 64, 16, 4, 2, 1),    # C3 / C5 shards
]
FALLBACK = [(8, 0, 128, 8, 256, 4, 4, 2, 1), (8, 1, 512, 2, 256, 4, 4, 2, 1)]  # 256 / 512 small-grid channels


def _ids(g):
    return "T" * g[1] + f"n{g[0]}-{g[2]}x{g[3]}-{g[4]}x{g[5]}k{g[6]}"


def _case(geom, xf, with_ep, seed):
    from cvhip import _lib

    n, tr, cin, hin, cout, hout, k, s, p = geom
    dev = torch.device("cuda")
    rng = np.random.default_rng(seed)
    op = (hout - ((hin - 1) * s - 2 * p + k)) if tr else 0
    g = _lib.cv_conv(n, cin, hin, hin, cout, hout, hout, k, k, s, p, tr)
    wshape = (cin, cout, k, k) if tr else (cout, cin, k, k)
    W = torch.tensor(rng.uniform(-0.2, 0.2, wshape), dtype=torch.float32, device=dev)
    Wf, Wb = _packed(_lib, W, tr)
    gat = Wb if tr else Wf  # the `gather` packing Wg[tap][cb][cs]
    s_ = _lib.stream_handle()
    if tr:  # ConvTranspose2d forward: small = input [n, hin, hin, cin], big = output
        cs, hs, cb, hb = cin, hin, cout, hout
    else:  # Conv2d backward-data: small = dY [n, hout, hout, cout], big = dX
        cs, hs, cb, hb = cout, hout, cin, hin
    x = torch.tensor(rng.standard_normal((n, hs, hs, cs)), dtype=torch.float32, device=dev)
    rm_s, rv_s = torch.zeros(cs, device=dev), torch.ones(cs, device=dev)
    if xf == "none":
        opnd = _lib.cv_operand(x.data_ptr(), None, _lib.XF_NONE, 0)
        a_host = x.double().cpu()
    elif tr:  # BN + ReLU of the layer below (ConvT input)
        gi, bi = _bn_state(cs, n * hs * hs, rng, dev)
        st = _stats_of(x, cs)
        opnd = _lib.cv_operand(x.data_ptr(), None, _lib.XF_BNRELU, 0, _cvbn(_lib, gi, bi, st, None, cs, n * hs * hs,
                                                                              rm_s, rv_s))
        a_host = _host_bnrelu(x, gi, bi, cs).cpu()
    else:  # BN backward of the conv output's BatchNorm (dY = BNbwd(dz))
        yo = torch.tensor(rng.standard_normal((n, hs, hs, cs)) * 2 + 0.5, dtype=torch.float32, device=dev)
        go, bo = _bn_state(cs, n * hs * hs, rng, dev)
        st = _stats_of(yo, cs)
        gst = torch.zeros(_lib.stat_repl(cs), 2, cs, dtype=torch.float64, device=dev)
        v = yo.double().reshape(-1, cs)
        xh = (v - v.mean(0)) / torch.sqrt(v.var(0, unbiased=False) + 1e-5)
        gst[0, 0] = x.double().reshape(-1, cs).sum(0)
        gst[0, 1] = (x.double().reshape(-1, cs) * xh).sum(0)
        opnd = _lib.cv_operand(x.data_ptr(), yo.data_ptr(), _lib.XF_BNBWD, 0,
                               _cvbn(_lib, go, bo, st, gst, cs, n * hs * hs, rm_s, rv_s))
        a_host = _host_bnbwd(x, yo, go, cs).cpu()
    a_nchw = a_host.permute(0, 3, 1, 2)
    Wd = W.double().cpu()
    b = torch.tensor(rng.uniform(-0.2, 0.2, cout), dtype=torch.float32, device=dev) if tr else None
    if tr:
        ref = F.conv_transpose2d(a_nchw, Wd, b.double().cpu(), stride=s, padding=p, output_padding=op)
    else:
        ref = torch.nn.grad.conv2d_input((n, cin, hin, hin), Wd, a_nchw, stride=s, padding=p)
    ref = ref.permute(0, 2, 3, 1).reshape(-1, cb)
    # epilogue: ConvT forward -> STAT_FWD of its BatchNorm; Conv2d backward-data -> STAT_BWD of the BN below
    ep = _lib.cv_epilogue()
    sums = None
    if with_ep:
        sums = torch.zeros(_lib.stat_repl(cb), 2, cb, dtype=torch.float64, device=dev)
        ep.stat_out, ep.stat_div = sums.data_ptr(), 1
        if tr:
            ep.stat_mode = _lib.STAT_FWD
            want = (ref.sum(0), (ref * ref).sum(0))
        else:
            yin = torch.tensor(rng.standard_normal((n, hb, hb, cb)) * 1.5 + 0.3, dtype=torch.float32, device=dev)
            ge, be = _bn_state(cb, n * hb * hb, rng, dev)
            rm_b, rv_b = torch.zeros(cb, device=dev), torch.ones(cb, device=dev)
            ep.stat_mode = _lib.STAT_BWD
            ep.ey = yin.data_ptr()
            st_b = _stats_of(yin, cb)  # (kept alive: the struct holds raw pointers)
            ep.ebn = _cvbn(_lib, ge, be, st_b, sums, cb, n * hb * hb, rm_b, rv_b)
            ep.erelu = 1
            vv = yin.double().cpu().reshape(-1, cb)
            xhb = (vv - vv.mean(0)) / torch.sqrt(vv.var(0, unbiased=False) + 1e-5)
            act = xhb * ge.double().cpu() + be.double().cpu()
            ref = ref * (act > 0)
            want = (ref.sum(0), (ref * xhb).sum(0))
    outs = {}
    for kind in ("direct", "core"):
        out = torch.full((n, hb, hb, cb), 7.0, dtype=torch.float32, device=dev)
        if sums is not None:
            sums.zero_()
        _lib.lib().cv_debug_direct_count(1)
        if kind == "direct":
            if tr:
                _lib.call("cv_conv_forward_kpack", g, opnd, Wf.data_ptr(), gat.data_ptr(), b.data_ptr(), out.data_ptr(),
                          ep, s_)
            else:
                _lib.call("cv_conv_backward_data_kpack", g, opnd, Wb.data_ptr(), gat.data_ptr(), out.data_ptr(), ep, s_)
        else:
            if tr:
                _lib.call("cv_conv_forward", g, opnd, Wf.data_ptr(), b.data_ptr(), out.data_ptr(), ep, s_)
            else:
                _lib.call("cv_conv_backward_data", g, opnd, Wb.data_ptr(), out.data_ptr(), ep, s_)
        torch.cuda.synchronize()
        launches = _lib.lib().cv_debug_direct_count(1)
        outs[kind] = (out.reshape(-1, cb).clone(), None if sums is None else sums.sum(0).cpu().clone(), launches)
    return outs, ref, (want if sums is not None else None)


@pytest.mark.parametrize("geom", SERVED, ids=_ids)
@pytest.mark.parametrize("xf,with_ep", [("none", False), ("bn", True)])
def test_direct_scatter(geom, xf, with_ep):
    outs, ref, want = _case(geom, xf, with_ep, 11 + sum(geom))
    d, c = outs["direct"], outs["core"]
    assert d[2] == 1 and c[2] == 0, ("direct kernel launches", d[2], c[2])
    assert rel(d[0], ref) < TOL, ("direct vs fp64", rel(d[0], ref))
    assert rel(d[0], c[0]) < 2e-6, ("direct vs GEMM core", rel(d[0], c[0]))
    if want is not None:
        assert rel(d[1][0], want[0]) < 1e-5 and rel(d[1][1], want[1]) < 1e-5, (rel(d[1][0], want[0]),
                                                                                rel(d[1][1], want[1]))


@pytest.mark.parametrize("geom", FALLBACK, ids=_ids)
def test_direct_scatter_fallback(geom):
    outs, ref, want = _case(geom, "bn", True, 5)
    d = outs["direct"]
    assert d[2] == 0, "the direct kernel does not serve > 128 small-grid channels"
    assert rel(d[0], ref) < TOL
    assert rel(d[1][0], want[0]) < 1e-5 and rel(d[1][1], want[1]) < 1e-5
