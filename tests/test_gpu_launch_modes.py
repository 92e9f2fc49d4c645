"""Full-batch parity of the GEMM core's launch modes (cv_gemm.hpp): the two-tile launch (gemm_kernel2, used when
a GATHER / SCATTER launch has more tiles than one round of resident slots) and the 4-deep operand ring (used
when a launch fills less than half a round).  The kernel tests in test_gpu_conv_kernels.py run at n = 8..64,
where every launch is under-filled; these run the geometries the bench runs at their full batch:

  * MNIST encoder conv2 backward-data at n = 512 with the BN-backward operand transform and the STAT_BWD
    epilogue (the bench's dominant call `enc[4]`: 1568 tiles, two-tile launch);
  * VAE64 encoder conv2 backward-data at n = 256 (4096 tiles: two-tile launch over several rounds);
  * the VAE64 conv5 forward at n = 32 (the PACS shard: under-filled, deep ring) and n = 256.

Reference: fp64 torch-CPU of the same math, tolerance 1e-5 rel-L2 (as test_gpu_conv_kernels.py)."""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from test_gpu_conv_kernels import TOL, _bn_state, _cvbn, _host_bnbwd, _host_bnrelu, _packed, _stats_of, rel

pytestmark = pytest.mark.gpu

# (n, transposed, c_in, h_in, c_out, h_out, k, s, p)
BWD = [(512, 0, 32, 14, 64, 7, 3, 2, 1), (256, 0, 32, 32, 64, 16, 4, 2, 1),
       # tile counts between the one-tile and the two-tile entries' resident slots (and below both), where
       # the two-tile grid is clamped to the tile count: MNIST conv2 at n = 256 (~784 tiles), VAE64 conv2 at
       # n = 128 / 64
       (256, 0, 32, 14, 64, 7, 3, 2, 1), (128, 0, 32, 32, 64, 16, 4, 2, 1), (64, 0, 32, 32, 64, 16, 4, 2, 1),
       (384, 0, 32, 14, 64, 7, 3, 2, 1)]
FWD = [(32, 0, 256, 4, 512, 2, 4, 2, 1), (256, 0, 256, 4, 512, 2, 4, 2, 1), (256, 1, 64, 16, 32, 32, 4, 2, 1)]


def _ids(g):
    return f"n{g[0]}-{'T' * g[1]}{g[2]}x{g[3]}-{g[4]}x{g[5]}"


@pytest.mark.parametrize("geom", BWD, ids=_ids)
def test_backward_data_bnbwd_statbwd_full_batch(geom):
    """dx of a conv whose output gradient passes the BN backward (operand transform), with the STAT_BWD
    epilogue of the BN+ReLU that feeds the conv: stored dz = dx * [active], sums (dz, dz * xhat)."""
    from cvhip import _lib

    n, tr, cin, hin, cout, hout, k, s, p = geom
    dev = torch.device("cuda")
    rng = np.random.default_rng(11 + n + cin)
    g = _lib.cv_conv(n, cin, hin, hin, cout, hout, hout, k, k, s, p, tr)
    W = torch.tensor(rng.uniform(-0.2, 0.2, (cout, cin, k, k)), dtype=torch.float32, device=dev)
    dzo = torch.tensor(rng.standard_normal((n, hout, hout, cout)), dtype=torch.float32, device=dev)
    yo = torch.tensor(rng.standard_normal((n, hout, hout, cout)) * 2 + 0.5, dtype=torch.float32, device=dev)
    yin = torch.tensor(rng.standard_normal((n, hin, hin, cin)) * 1.5 + 0.3, dtype=torch.float32, device=dev)
    # operand: BN backward of the conv's output BN layer
    go_, bo_ = _bn_state(cout, n * hout * hout, rng, dev)
    st_o = _stats_of(yo, cout)
    gst_o = torch.zeros(_lib.stat_repl(cout), 2, cout, dtype=torch.float64, device=dev)
    v = yo.double().reshape(-1, cout)
    xh_o = (v - v.mean(0)) / torch.sqrt(v.var(0, unbiased=False) + 1e-5)
    gst_o[0, 0] = dzo.double().reshape(-1, cout).sum(0)
    gst_o[0, 1] = (dzo.double().reshape(-1, cout) * xh_o).sum(0)
    rm_o, rv_o = torch.zeros(cout, device=dev), torch.ones(cout, device=dev)
    gop = _lib.cv_operand(dzo.data_ptr(), yo.data_ptr(), _lib.XF_BNBWD, 0,
                          _cvbn(_lib, go_, bo_, st_o, gst_o, cout, n * hout * hout, rm_o, rv_o))
    # epilogue: the BN+ReLU of the conv's input
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
    _, Wb = _packed(_lib, W, tr)
    _lib.call("cv_conv_backward_data", g, gop, Wb.data_ptr(), gin.data_ptr(), ep, _lib.stream_handle())
    dy_nchw = _host_bnbwd(dzo, yo, go_, cout).permute(0, 3, 1, 2).cpu()
    gref = torch.nn.grad.conv2d_input((n, cin, hin, hin), W.double().cpu(), dy_nchw, stride=s, padding=p)
    gref = gref.permute(0, 2, 3, 1).reshape(-1, cin)
    vi = yin.double().cpu().reshape(-1, cin)
    xh = (vi - vi.mean(0)) / torch.sqrt(vi.var(0, unbiased=False) + 1e-5)
    dz = gref * ((xh * gi.double().cpu() + bi.double().cpu()) > 0)
    torch.cuda.synchronize()
    assert rel(gin.reshape(-1, cin), dz) < TOL, rel(gin.reshape(-1, cin), dz)
    sums = gst.sum(0).cpu()
    assert rel(sums[0], dz.sum(0)) < 1e-5
    assert rel(sums[1], (dz * xh).sum(0)) < 1e-5


@pytest.mark.parametrize("geom", FWD, ids=_ids)
def test_forward_bnrelu_statfwd_full_batch(geom):
    """Forward conv / convT with the BN+ReLU operand transform and the STAT_FWD epilogue."""
    from cvhip import _lib

    n, tr, cin, hin, cout, hout, k, s, p = geom
    dev = torch.device("cuda")
    rng = np.random.default_rng(23 + n + cin)
    g = _lib.cv_conv(n, cin, hin, hin, cout, hout, hout, k, k, s, p, tr)
    wshape = (cin, cout, k, k) if tr else (cout, cin, k, k)
    W = torch.tensor(rng.uniform(-0.2, 0.2, wshape), dtype=torch.float32, device=dev)
    b = torch.tensor(rng.uniform(-0.2, 0.2, cout), dtype=torch.float32, device=dev)
    x = torch.tensor(rng.standard_normal((n, hin, hin, cin)), dtype=torch.float32, device=dev)
    gi, bi = _bn_state(cin, n * hin * hin, rng, dev)
    rm, rv = torch.zeros(cin, device=dev), torch.ones(cin, device=dev)
    st_i = _stats_of(x, cin)  # (kept alive: the struct below only holds its device pointer)
    opnd = _lib.cv_operand(x.data_ptr(), None, _lib.XF_BNRELU, 0,
                           _cvbn(_lib, gi, bi, st_i, None, cin, n * hin * hin, rm, rv))
    out = torch.empty(n, hout, hout, cout, dtype=torch.float32, device=dev)
    ep = _lib.cv_epilogue()
    ep.stat_mode, ep.stat_div = _lib.STAT_FWD, 1
    st_out = torch.zeros(_lib.stat_repl(cout), 2, cout, dtype=torch.float64, device=dev)
    ep.stat_out = st_out.data_ptr()
    Wf, _ = _packed(_lib, W, tr)
    _lib.call("cv_conv_forward", g, opnd, Wf.data_ptr(), b.data_ptr(), out.data_ptr(), ep, _lib.stream_handle())
    xin = _host_bnrelu(x, gi, bi, cin).permute(0, 3, 1, 2).cpu()
    Wd, bd = W.double().cpu(), b.double().cpu()
    if tr:
        op = hout - ((hin - 1) * s - 2 * p + k)
        ref = F.conv_transpose2d(xin, Wd, bd, stride=s, padding=p, output_padding=op)
    else:
        ref = F.conv2d(xin, Wd, bd, stride=s, padding=p)
    ref = ref.permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    assert rel(out, ref) < TOL, rel(out, ref)
    ssum = st_out.sum(0).cpu()
    assert rel(ssum[0], ref.reshape(-1, cout).sum(0)) < 1e-6
    assert rel(ssum[1], (ref.reshape(-1, cout) ** 2).sum(0)) < 1e-6
