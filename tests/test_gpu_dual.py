"""The dual launch (csrc/cv_dual.hip): cv_conv_backward_deferred_kpack issues a served layer's backward-data (direct
kernel) and its weight gradient (GEMM-core WGRAD) as ONE grid whose workgroups alternate roles.  For each pair the
MNIST bench serves at n = 512 (vae.py:15-46: conv2 / conv3 backward-data SCATTER, convT2 backward-data GATHER) the
call runs twice on the same operands — dual grid on (the default) and off (cv_debug_dual(0): the two launches back
to back) — and:
  * the dual grid really ran (cv_debug_dual_count) and did not run with it off;
  * the data gradient is bit-identical (the direct role's arithmetic does not depend on the grid it runs in);
  * the BatchNorm-backward sums of the STAT_BWD epilogue agree to 1e-12 (fp64 atomics, arrival order varies) and
    the constants the last direct workgroup finalises (cbwd = [sc][c1][mu][istd][c2], counted over the direct
    role's own workgroups, bn_finalize_at) agree to 2e-6 and with a host fold of those sums;
  * the deferred weight-gradient partials, reduced by cv_step_reduce, agree to 2e-6 (the dual grid takes 64-row
    WGRAD tiles, dual_wgrad_bm_cap, so the split can differ; bit-identical when the plans coincide);
  * both agree with fp64 torch (data gradient with the ReLU mask of the layer below, weight gradient) at 1e-5."""

import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from test_gpu_conv_kernels import TOL, _host_bnbwd, _host_bnrelu, _packed, rel

pytestmark = pytest.mark.gpu

# (n, transposed, c_in, h_in, c_out, h_out, k, s, p)
PAIRS = {
    "mnist_conv2": (512, 0, 32, 14, 64, 7, 3, 2, 1),
    "mnist_conv3": (512, 0, 64, 7, 128, 4, 3, 2, 1),
    "mnist_convT2": (512, 1, 64, 7, 32, 14, 3, 2, 1),
}


def _bn(lib, C, count, rng, dev, y=None, gsum=None):
    """A train-mode BatchNorm descriptor: forward sums of y (fp64 replica 0), optional backward sums, ticket and
    finalised-constant buffers."""
    t = dict(gamma=torch.tensor(rng.uniform(0.5, 1.5, C), dtype=torch.float32, device=dev),
             beta=torch.tensor(rng.uniform(-0.3, 0.3, C), dtype=torch.float32, device=dev),
             stat=torch.zeros(lib.stat_repl(C), 2, C, dtype=torch.float64, device=dev),
             gstat=torch.zeros(lib.stat_repl(C), 2, C, dtype=torch.float64, device=dev),
             rm=torch.zeros(C, device=dev), rv=torch.ones(C, device=dev),
             cfwd=torch.zeros(4 * C, device=dev), cbwd=torch.zeros(5 * C, device=dev),
             ticket=torch.zeros(lib.TICKET_WORDS, dtype=torch.int32, device=dev))
    v = y.double().reshape(-1, C)
    t["stat"][0, 0] = v.sum(0)
    t["stat"][0, 1] = (v * v).sum(0)
    if gsum is not None:
        t["gstat"][0] = gsum
    s = lib.cv_bn(t["gamma"].data_ptr(), t["beta"].data_ptr(), t["stat"].data_ptr(), t["gstat"].data_ptr(),
                  t["rm"].data_ptr(), t["rv"].data_ptr(), C, count, 1, 1e-5, t["cfwd"].data_ptr(),
                  t["cbwd"].data_ptr(), t["ticket"].data_ptr())
    return s, t


def _run(name, dual, self_reduce=None):
    from cvhip import _lib

    n, tr, cin, hin, cout, hout, k, s, p = PAIRS[name]
    dev = torch.device("cuda")
    L = _lib.lib()
    rng = np.random.default_rng(sum(PAIRS[name]))
    g = _lib.cv_conv(n, cin, hin, hin, cout, hout, hout, k, k, s, p, tr)
    W = torch.tensor(rng.uniform(-0.2, 0.2, (cin, cout, k, k) if tr else (cout, cin, k, k)), dtype=torch.float32,
                     device=dev)
    Wf, Wb = _packed(_lib, W, tr)
    # the layer input (pre-BN values of the BatchNorm below: BN + ReLU on load, and the STAT_BWD epilogue's mask)
    x = torch.tensor(rng.standard_normal((n, hin, hin, cin)) * 1.5 + 0.3, dtype=torch.float32, device=dev)
    bin_, tin = _bn(_lib, cin, n * hin * hin, rng, dev, y=x)
    # the output gradient dz and the output's pre-BN values (BN backward on load)
    dz = torch.tensor(rng.standard_normal((n, hout, hout, cout)), dtype=torch.float32, device=dev)
    yo = torch.tensor(rng.standard_normal((n, hout, hout, cout)) * 2 + 0.5, dtype=torch.float32, device=dev)
    vo = yo.double().reshape(-1, cout)
    xh = (vo - vo.mean(0)) / torch.sqrt(vo.var(0, unbiased=False) + 1e-5)
    gsum = torch.stack([dz.double().reshape(-1, cout).sum(0), (dz.double().reshape(-1, cout) * xh).sum(0)])
    bout, tout = _bn(_lib, cout, n * hout * hout, rng, dev, y=yo, gsum=gsum)
    gout = _lib.cv_operand(dz.data_ptr(), yo.data_ptr(), _lib.XF_BNBWD, 0, bout)
    xin = _lib.cv_operand(x.data_ptr(), None, _lib.XF_BNRELU, 0, bin_)
    ep = _lib.cv_epilogue()
    ep.stat_mode = _lib.STAT_BWD
    ep.stat_out = tin["gstat"].data_ptr()
    ep.stat_div = 1
    ep.ey = x.data_ptr()
    ep.ebn = bin_
    ep.erelu = 1
    gin = torch.full((n, hin, hin, cin), 7.0, device=dev)
    gw = torch.zeros(W.shape, device=dev)
    wb = int(L.cv_conv_wgrad_workspace_bytes(ctypes.byref(g), 0))
    work = torch.full((wb // 4 + 4,), 3.0, device=dev)
    d = _lib.cv_wgrad_defer()
    st = _lib.stream_handle()
    prev = L.cv_debug_dual(1 if dual else 0)
    prev_self = L.cv_debug_wgrad_self(-1 if self_reduce is None else int(self_reduce))
    L.cv_debug_dual_count(1)
    try:
        _lib.call("cv_conv_backward_deferred_kpack", ctypes.byref(g), ctypes.byref(gout), Wb.data_ptr(),
                  Wf.data_ptr(), gin.data_ptr(), ctypes.byref(ep), ctypes.byref(xin), gw.data_ptr(), None,
                  work.data_ptr(), work.numel() * 4, ctypes.byref(d), st)
        torch.cuda.synchronize()
        issued = L.cv_debug_dual_count(1)
    finally:
        L.cv_debug_dual(prev)
        if self_reduce is not None:
            L.cv_debug_wgrad_self(prev_self)
    # (two forms: the split's partials recorded for cv_step_reduce (the default), or — the opt-in self-reducing
    # split — the split's last slice already added the gradient and the record says split 0)
    parts = None
    if d.split > 0:
        assert d.part == work.data_ptr()
        parts = work[: d.split * d.M * d.ntot].clone()
        _lib.call("cv_step_reduce", (_lib.cv_wgrad_defer * 1)(d), 1, None, 0, None, None, 0, ctypes.c_float(0.1),
                  None, st)
        torch.cuda.synchronize()
    host = dict(x=x, dz=dz, yo=yo, W=W, tin=tin, tout=tout, geom=PAIRS[name])
    return dict(issued=issued, gin=gin.clone(), gsum=tin["gstat"].sum(0).cpu(), cbwd=tin["cbwd"].cpu(),
                ticket=int(tin["ticket"][1].item()), split=(d.split, d.M, d.ntot), parts=parts, gw=gw.clone(),
                host=host)


def _fp64(h):
    """fp64 data gradient (masked by the ReLU of the BatchNorm below) and weight gradient of the layer."""
    n, tr, cin, hin, cout, hout, k, s, p = h["geom"]
    a = _host_bnrelu(h["x"], h["tin"]["gamma"], h["tin"]["beta"], cin).cpu()
    go = _host_bnbwd(h["dz"], h["yo"], h["tout"]["gamma"], cout).cpu()
    a_ = a.permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    w_ = h["W"].double().cpu().requires_grad_(True)
    if tr:
        op = hout - ((hin - 1) * s - 2 * p + k)
        y = F.conv_transpose2d(a_, w_, stride=s, padding=p, output_padding=op)
    else:
        y = F.conv2d(a_, w_, stride=s, padding=p)
    y.backward(go.permute(0, 3, 1, 2))
    v = h["x"].double().cpu().reshape(-1, cin)
    act = (v - v.mean(0)) / torch.sqrt(v.var(0, unbiased=False) + 1e-5) * h["tin"]["gamma"].double().cpu() + \
        h["tin"]["beta"].double().cpu()
    gin = a_.grad.permute(0, 2, 3, 1).reshape(-1, cin) * (act > 0)
    return gin, w_.grad, v


@pytest.mark.parametrize("name", list(PAIRS))
def test_dual_grid_matches_back_to_back(name):
    on, off = _run(name, True), _run(name, False)
    assert on["issued"] == 1, "the served pair did not run as one dual grid"
    assert off["issued"] == 0
    assert torch.equal(on["gin"], off["gin"]), "data gradient differs between the dual grid and the direct launch"
    gs_on, gs_off = on["gsum"], off["gsum"]
    assert float((gs_on - gs_off).abs().max()) <= 1e-12 * max(1.0, float(gs_off.abs().max()))
    # the finalised BN-backward constants: both runs' last direct workgroup wrote them, and they fold the sums
    assert on["ticket"] != 0 and off["ticket"] != 0, "the direct role's BatchNorm finalisation did not run"
    assert on["ticket"] == off["ticket"], "the dual grid counted other than the direct role's own workgroups"
    assert rel(on["cbwd"], off["cbwd"]) < 2e-6
    h = on["host"]
    n, tr, cin, hin, cout, hout, k, s, p = h["geom"]
    cnt = n * hin * hin
    c1 = gs_on[0] / cnt
    c2 = gs_on[1] / cnt
    assert rel(on["cbwd"][cin:2 * cin], c1) < 1e-6 and rel(on["cbwd"][4 * cin:5 * cin], c2) < 1e-6
    # weight gradient: partials bit-identical when both plans coincide, reduced gradients within 2e-6 always
    if on["split"] == off["split"] and on["parts"] is not None:
        assert torch.equal(on["parts"], off["parts"])
    assert rel(on["gw"], off["gw"]) < 2e-6, rel(on["gw"], off["gw"])
    # both against fp64
    gin_ref, gw_ref, v = _fp64(h)
    assert rel(on["gin"].reshape(-1, cin), gin_ref) < TOL
    assert rel(on["gw"], gw_ref) < TOL, rel(on["gw"], gw_ref)
    xh = (v - v.mean(0)) / torch.sqrt(v.var(0, unbiased=False) + 1e-5)
    want = torch.stack([gin_ref.sum(0), (gin_ref * xh).sum(0)])
    assert rel(gs_on, want) < 1e-5


@pytest.mark.parametrize("name", list(PAIRS))
@pytest.mark.parametrize("dual", [True, False], ids=["dual", "back-to-back"])
def test_self_reducing_wgrad_matches_step_reduce(name, dual):
    """The deferred weight gradient reduced by its own last slice (cv_debug_wgrad_self(1), opt-in) against the
    same partials summed by cv_step_reduce (0): the same slabs in the same slice order, added by another kernel's
    association — within 2e-6 — and both against fp64 at 1e-5; the data gradient is unaffected (bit-identical)."""
    a, b = _run(name, dual, True), _run(name, dual, False)
    assert a["split"][0] == 0 and b["split"][0] > 1, (a["split"], b["split"])
    assert torch.equal(a["gin"], b["gin"])
    assert rel(a["gw"], b["gw"]) < 2e-6, rel(a["gw"], b["gw"])
    gin_ref, gw_ref, _ = _fp64(a["host"])
    assert rel(a["gw"], gw_ref) < TOL, rel(a["gw"], gw_ref)
