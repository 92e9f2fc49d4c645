"""The direct stride-2 conv kernel (cv_direct.hip, reached through cv_conv_forward_kpack /
cv_conv_backward_data_kpack): both contraction shapes at every stride-2 geometry of VAE and VAE64 it serves
(vae.py:15-46, 113-156) —
  * SCATTER (class-fused: Conv2d backward-data, ConvTranspose2d forward),
  * GATHER (parity-plane region: Conv2d forward, ConvTranspose2d backward-data),
with and without the fused BatchNorm transforms and statistics epilogues, at small, ragged and the benches' full
batches.

Each case is checked three ways:
  * the direct kernel really ran (cv_debug_direct_count), or — for the geometries it does not serve (VAE64's
    256 / 512-channel operands, grids under 256 workgroups) — the kpack call fell back to the GEMM core;
  * against an fp64 torch evaluation of the same math at the kernel bar 1e-5 (tests/test_gpu_conv_kernels.py),
    including the epilogue's fp64 batch sums;
  * against the implicit-GEMM core on the same operands (the calls without kpack): the same contraction summed
    in another order, so within 2e-6 relative."""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from test_gpu_conv_kernels import TOL, _bn_state, _cvbn, _host_bnbwd, _host_bnrelu, _packed, _stats_of, rel

pytestmark = pytest.mark.gpu

# (n, transposed, c_in, h_in, c_out, h_out, k, s, p)
LAYERS = {
    "mnist_conv2": (32, 0, 32, 14, 64, 7, 3, 2, 1), "mnist_conv3": (32, 0, 64, 7, 128, 4, 3, 2, 1),
    "mnist_convT1": (32, 1, 128, 4, 64, 7, 3, 2, 1), "mnist_convT2": (32, 1, 64, 7, 32, 14, 3, 2, 1),
    "v64_conv2": (8, 0, 32, 32, 64, 16, 4, 2, 1), "v64_conv3": (8, 0, 64, 16, 128, 8, 4, 2, 1),
    "v64_conv4": (8, 0, 128, 8, 256, 4, 4, 2, 1),
    "v64_convT2": (8, 1, 256, 4, 128, 8, 4, 2, 1), "v64_convT3": (8, 1, 128, 8, 64, 16, 4, 2, 1),
    "v64_convT4": (8, 1, 64, 16, 32, 32, 4, 2, 1),
}


def _with_n(name, n):
    return (n,) + LAYERS[name][1:]


# (geometry, direction) pairs the direct kernel serves: the staged operand has <= 128 channels
SERVED = [(LAYERS[k], d) for k in LAYERS for d in ("fwd", "bwd")
          if (LAYERS[k][2] if (d == "fwd") else LAYERS[k][4]) <= 128]
SERVED += [(_with_n("mnist_conv2", 5), "bwd"), (_with_n("v64_convT3", 3), "fwd"), (_with_n("mnist_conv2", 7), "fwd"),
           (_with_n("v64_convT3", 3), "bwd"),                                              # ragged batches
           (_with_n("mnist_conv2", 512), "bwd"), (_with_n("mnist_conv2", 512), "fwd"),     # the MNIST bench batch
           (_with_n("mnist_convT2", 512), "fwd"), (_with_n("mnist_convT2", 512), "bwd"),
           (_with_n("v64_conv2", 256), "bwd"), (_with_n("v64_conv2", 256), "fwd"),         # C3 / C5 shards
           (_with_n("v64_convT3", 128), "fwd"), (_with_n("v64_conv3", 128), "fwd")]
NOT_SERVED = [(LAYERS["v64_conv4"], "bwd"), (LAYERS["v64_convT2"], "fwd")]  # 256 staged channels
UNDERFILLED = [(_with_n("v64_conv3", 32), "bwd")]  # the C4 shard's conv3: 128 workgroups at most -> GEMM core


def _ids(v):
    g, d = v
    return f"{d}-" + "T" * g[1] + f"n{g[0]}-{g[2]}x{g[3]}-{g[4]}x{g[5]}k{g[6]}"


@pytest.fixture(autouse=True)
def _any_grid():
    """The kernel-level cases run the direct kernel at any grid size and any GATHER tile (the product falls back
    to the GEMM core below 256 workgroups, cv_debug_direct_minwg, and for the GATHER geometries where the core
    measured faster, cv_debug_direct_gather_rule); restored afterwards."""
    from cvhip import _lib

    prev = _lib.lib().cv_debug_direct_minwg(1)
    prev_rule = _lib.lib().cv_debug_direct_gather_rule(0)
    yield
    _lib.lib().cv_debug_direct_minwg(prev)  # (-1: re-read CV_DIRECT_MINWG / the default)
    _lib.lib().cv_debug_direct_gather_rule(prev_rule)


def _case(geom, direction, with_xf, seed):
    """Run the contraction through the kpack call and through the plain call; returns both and the fp64 refs."""
    from cvhip import _lib

    n, tr, cin, hin, cout, hout, k, s, p = geom
    dev = torch.device("cuda")
    rng = np.random.default_rng(seed)
    op = (hout - ((hin - 1) * s - 2 * p + k)) if tr else 0
    g = _lib.cv_conv(n, cin, hin, hin, cout, hout, hout, k, k, s, p, tr)
    wshape = (cin, cout, k, k) if tr else (cout, cin, k, k)
    W = torch.tensor(rng.uniform(-0.2, 0.2, wshape), dtype=torch.float32, device=dev)
    Wf, Wb = _packed(_lib, W, tr)
    s_ = _lib.stream_handle()
    fwd = direction == "fwd"
    # staged operand: the layer input (forward) or the output gradient (backward-data)
    ca, ha, cz, hz = (cin, hin, cout, hout) if fwd else (cout, hout, cin, hin)
    x = torch.tensor(rng.standard_normal((n, ha, ha, ca)), dtype=torch.float32, device=dev)
    rm_a, rv_a = torch.zeros(ca, device=dev), torch.ones(ca, device=dev)
    keep = []
    if not with_xf:
        opnd = _lib.cv_operand(x.data_ptr(), None, _lib.XF_NONE, 0)
        a_host = x.double().cpu()
    elif fwd:  # BN + ReLU of the layer below
        gi, bi = _bn_state(ca, n * ha * ha, rng, dev)
        st = _stats_of(x, ca)
        keep += [gi, bi, st]
        opnd = _lib.cv_operand(x.data_ptr(), None, _lib.XF_BNRELU, 0, _cvbn(_lib, gi, bi, st, None, ca, n * ha * ha,
                                                                              rm_a, rv_a))
        a_host = _host_bnrelu(x, gi, bi, ca).cpu()
    else:  # BN backward of the layer output's BatchNorm
        yo = torch.tensor(rng.standard_normal((n, ha, ha, ca)) * 2 + 0.5, dtype=torch.float32, device=dev)
        go, bo = _bn_state(ca, n * ha * ha, rng, dev)
        st = _stats_of(yo, ca)
        gst = torch.zeros(_lib.stat_repl(ca), 2, ca, dtype=torch.float64, device=dev)
        v = yo.double().reshape(-1, ca)
        xh = (v - v.mean(0)) / torch.sqrt(v.var(0, unbiased=False) + 1e-5)
        gst[0, 0] = x.double().reshape(-1, ca).sum(0)
        gst[0, 1] = (x.double().reshape(-1, ca) * xh).sum(0)
        keep += [yo, go, bo, st, gst]
        opnd = _lib.cv_operand(x.data_ptr(), yo.data_ptr(), _lib.XF_BNBWD, 0,
                               _cvbn(_lib, go, bo, st, gst, ca, n * ha * ha, rm_a, rv_a))
        a_host = _host_bnbwd(x, yo, go, ca).cpu()
    a_nchw = a_host.permute(0, 3, 1, 2)
    Wd = W.double().cpu()
    b = torch.tensor(rng.uniform(-0.2, 0.2, cout), dtype=torch.float32, device=dev) if fwd else None
    if fwd and tr:
        ref = F.conv_transpose2d(a_nchw, Wd, b.double().cpu(), stride=s, padding=p, output_padding=op)
    elif fwd:
        ref = F.conv2d(a_nchw, Wd, b.double().cpu(), stride=s, padding=p)
    elif tr:
        ref = F.conv2d(a_nchw, Wd, None, stride=s, padding=p)
    else:
        ref = torch.nn.grad.conv2d_input((n, cin, hin, hin), Wd, a_nchw, stride=s, padding=p)
    ref = ref.permute(0, 2, 3, 1).reshape(-1, cz)
    # epilogue: forward -> STAT_FWD of the output's BatchNorm; backward-data -> STAT_BWD of the BN below
    ep = _lib.cv_epilogue()
    sums, want = None, None
    if with_xf:
        sums = torch.zeros(_lib.stat_repl(cz), 2, cz, dtype=torch.float64, device=dev)
        ep.stat_out, ep.stat_div = sums.data_ptr(), 1
        if fwd:
            ep.stat_mode = _lib.STAT_FWD
            want = (ref.sum(0), (ref * ref).sum(0))
        else:
            yin = torch.tensor(rng.standard_normal((n, hz, hz, cz)) * 1.5 + 0.3, dtype=torch.float32, device=dev)
            ge, be = _bn_state(cz, n * hz * hz, rng, dev)
            rm_b, rv_b = torch.zeros(cz, device=dev), torch.ones(cz, device=dev)
            st_b = _stats_of(yin, cz)
            keep += [yin, ge, be, rm_b, rv_b, st_b]
            ep.stat_mode = _lib.STAT_BWD
            ep.ey = yin.data_ptr()
            ep.ebn = _cvbn(_lib, ge, be, st_b, sums, cz, n * hz * hz, rm_b, rv_b)
            ep.erelu = 1
            vv = yin.double().cpu().reshape(-1, cz)
            xhb = (vv - vv.mean(0)) / torch.sqrt(vv.var(0, unbiased=False) + 1e-5)
            act = xhb * ge.double().cpu() + be.double().cpu()
            ref = ref * (act > 0)
            want = (ref.sum(0), (ref * xhb).sum(0))
    outs = {}
    for kind in ("direct", "core"):
        out = torch.full((n, hz, hz, cz), 7.0, dtype=torch.float32, device=dev)
        if sums is not None:
            sums.zero_()
        _lib.lib().cv_debug_direct_count(1)
        if fwd:
            bp = b.data_ptr()
            if kind == "direct":
                _lib.call("cv_conv_forward_kpack", g, opnd, Wf.data_ptr(), Wb.data_ptr(), bp, out.data_ptr(), ep, s_)
            else:
                _lib.call("cv_conv_forward", g, opnd, Wf.data_ptr(), bp, out.data_ptr(), ep, s_)
        else:
            if kind == "direct":
                _lib.call("cv_conv_backward_data_kpack", g, opnd, Wb.data_ptr(), Wf.data_ptr(), out.data_ptr(), ep, s_)
            else:
                _lib.call("cv_conv_backward_data", g, opnd, Wb.data_ptr(), out.data_ptr(), ep, s_)
        torch.cuda.synchronize()
        launches = _lib.lib().cv_debug_direct_count(1)
        outs[kind] = (out.reshape(-1, cz).clone(), None if sums is None else sums.sum(0).cpu().clone(), launches)
    return outs, ref, want


@pytest.mark.parametrize("case", SERVED, ids=_ids)
@pytest.mark.parametrize("with_xf", [False, True], ids=["plain", "bn"])
def test_direct_conv(case, with_xf):
    geom, direction = case
    outs, ref, want = _case(geom, direction, with_xf, 11 + sum(geom) + (direction == "bwd"))
    d, c = outs["direct"], outs["core"]
    assert d[2] == 1 and c[2] == 0, ("direct kernel launches", d[2], c[2])
    assert rel(d[0], ref) < TOL, ("direct vs fp64", rel(d[0], ref))
    assert rel(d[0], c[0]) < 2e-6, ("direct vs GEMM core", rel(d[0], c[0]))
    if want is not None:
        assert rel(d[1][0], want[0]) < 1e-5 and rel(d[1][1], want[1]) < 1e-5, (rel(d[1][0], want[0]),
                                                                                rel(d[1][1], want[1]))


@pytest.mark.parametrize("case", NOT_SERVED + UNDERFILLED, ids=_ids)
def test_direct_conv_fallback(case):
    from cvhip import _lib

    geom, direction = case
    if case in UNDERFILLED:
        _lib.lib().cv_debug_direct_minwg(256)
    outs, ref, want = _case(geom, direction, True, 5)
    d = outs["direct"]
    assert d[2] == 0, "the direct kernel does not serve this call"
    assert rel(d[0], ref) < TOL
    assert rel(d[1][0], want[0]) < 1e-5 and rel(d[1][1], want[1]) < 1e-5


# the production choice for GATHER (cv_debug_direct_gather_rule 1): the MNIST bench's conv2 forward / convT2
# backward-data (49-pixel tiles, 512 workgroups) take the direct kernel; MNIST conv3 forward (16-pixel tiles) and
# the C3 shard's conv2 forward (1024 workgroups) run the GEMM core
GATHER_RULE = [((_with_n("mnist_conv2", 512), "fwd"), 1), ((_with_n("mnist_convT2", 512), "bwd"), 1),
               ((_with_n("mnist_conv3", 512), "fwd"), 0), ((_with_n("v64_conv2", 256), "fwd"), 0)]


@pytest.mark.parametrize("case,served", GATHER_RULE, ids=lambda v: _ids(v) if isinstance(v, tuple) else str(v))
def test_direct_gather_rule(case, served):
    from cvhip import _lib

    _lib.lib().cv_debug_direct_minwg(-1)
    _lib.lib().cv_debug_direct_gather_rule(1)
    geom, direction = case
    outs, ref, want = _case(geom, direction, True, 9)
    d = outs["direct"]
    assert d[2] == served, (d[2], served)
    assert rel(d[0], ref) < TOL
