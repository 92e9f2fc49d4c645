"""Pixel-major tiles of the GEMM core (csrc/cv_gemm_tile.inc, Args::pm): for the convs whose padding taps are a large
share of the (pixel, tap) pairs — VAE64's conv4 / conv5 and their mirrors convT1 / convT2 (vae.py:123-128, 141-146),
MNIST's conv3 / convT1 (vae.py:19-21, 38-40) — a tile holds one pixel of BM images (WGRAD: a K tile holds 32
images at one small pixel), so the taps (pixels) its rows read in the padding are the same for the whole tile and
its K loop skips them.

Each geometry runs the forward (with and without the BN+ReLU operand transform and its STAT_FWD epilogue), the
backward-data (with the BN-backward transform, and with the STAT_BWD epilogue) and the weight gradient (split-K
partials and the atomic form) twice — pixel-major tiles on (cv_debug_pm(1)) and off — and checks:
  * the pixel-major plan was really taken (cv_debug_pm_count) on, and not off;
  * both against fp64 torch at the kernel bar 1e-5 (tests/test_gpu_conv_kernels.py, reused as is);
  * forward and backward-data outputs bit-identical on / off where no K split is involved (the skipped products
    are exact zeros and the visited K tiles keep their order), and everything within 2e-6 otherwise."""

import numpy as np
import pytest
import torch

import test_gpu_conv_kernels as KT  # (a module import: its test functions are not collected here again)

pytestmark = pytest.mark.gpu

# (n, transposed, c_in, h_in, c_out, h_out, k, s, p): batches that are multiples of the 64-row tile
PM_GEOMS = [
    (64, 0, 128, 8, 256, 4, 4, 2, 1), (64, 0, 256, 4, 512, 2, 4, 2, 1),    # VAE64 conv4, conv5
    (64, 1, 512, 2, 256, 4, 4, 2, 1), (64, 1, 256, 4, 128, 8, 4, 2, 1),    # VAE64 convT1, convT2
    (128, 0, 256, 4, 512, 2, 4, 2, 1),                                      # conv5 at the C5 shard
    (64, 0, 64, 7, 128, 4, 3, 2, 1), (64, 1, 128, 4, 64, 7, 3, 2, 1),       # MNIST conv3, convT1
]


def _ids(g):
    return f"n{g[0]}-" + "T" * g[1] + f"{g[2]}x{g[3]}-{g[4]}x{g[5]}k{g[6]}"


@pytest.fixture
def pm_mode():
    from cvhip import _lib

    L = _lib.lib()
    prev = L.cv_debug_pm(-1)

    def set_(on):
        L.cv_debug_pm(on)
        L.cv_debug_pm_count(1)

    yield set_, L
    L.cv_debug_pm(1 if prev < 0 else prev)


@pytest.mark.parametrize("geom", PM_GEOMS, ids=_ids)
@pytest.mark.parametrize("xf", ["none", "bn"])
@pytest.mark.parametrize("pm", [1, 0], ids=["pm", "image-major"])
def test_pm_conv_vs_fp64(geom, xf, pm, pm_mode):
    set_, L = pm_mode
    set_(pm)
    KT.test_conv_fwd_bwd_wgrad(geom, xf, "core")
    used = L.cv_debug_pm_count(1)
    assert (used > 0) == bool(pm), ("pixel-major plans", used)


@pytest.mark.parametrize("geom", PM_GEOMS, ids=_ids)
@pytest.mark.parametrize("pm", [1, 0], ids=["pm", "image-major"])
def test_pm_backward_stat_epilogue(geom, pm, pm_mode):
    set_, L = pm_mode
    set_(pm)
    KT.test_backward_data_stat_epilogue(geom, "core", batch=geom[0])
    used = L.cv_debug_pm_count(1)
    assert (used > 0) == bool(pm), ("pixel-major plans", used)


def _run_all(geom, pm, set_):
    """forward, backward-data and weight gradient of one geometry with BN transforms; returns the outputs."""
    from cvhip import _lib
    from test_gpu_conv_kernels import _bn_state, _cvbn, _packed, _stats_of

    set_(pm)
    n, tr, cin, hin, cout, hout, k, s, p = geom
    dev = torch.device("cuda")
    rng = np.random.default_rng(sum(geom))
    g = _lib.cv_conv(n, cin, hin, hin, cout, hout, hout, k, k, s, p, tr)
    wshape = (cin, cout, k, k) if tr else (cout, cin, k, k)
    W = torch.tensor(rng.uniform(-0.2, 0.2, wshape), dtype=torch.float32, device=dev)
    x = torch.tensor(rng.standard_normal((n, hin, hin, cin)), dtype=torch.float32, device=dev)
    dz = torch.tensor(rng.standard_normal((n, hout, hout, cout)), dtype=torch.float32, device=dev)
    yo = torch.tensor(rng.standard_normal((n, hout, hout, cout)) * 2 + 0.5, dtype=torch.float32, device=dev)
    gi, bi = _bn_state(cin, n * hin * hin, rng, dev)
    go, bo = _bn_state(cout, n * hout * hout, rng, dev)
    rm_i, rv_i = torch.zeros(cin, device=dev), torch.ones(cin, device=dev)
    rm_o, rv_o = torch.zeros(cout, device=dev), torch.ones(cout, device=dev)
    st_i, st_o = _stats_of(x, cin), _stats_of(yo, cout)
    gst = torch.zeros(_lib.stat_repl(cout), 2, cout, dtype=torch.float64, device=dev)
    gst[0, 0] = dz.double().reshape(-1, cout).sum(0)
    gst[0, 1] = dz.double().reshape(-1, cout).abs().sum(0) * 0.01
    opnd = _lib.cv_operand(x.data_ptr(), None, _lib.XF_BNRELU, 0,
                           _cvbn(_lib, gi, bi, st_i, None, cin, n * hin * hin, rm_i, rv_i))
    gop = _lib.cv_operand(dz.data_ptr(), yo.data_ptr(), _lib.XF_BNBWD, 0,
                          _cvbn(_lib, go, bo, st_o, gst, cout, n * hout * hout, rm_o, rv_o))
    Wf, Wb = _packed(_lib, W, tr)
    s_ = _lib.stream_handle()
    out = torch.empty(n, hout, hout, cout, device=dev)
    _lib.call("cv_conv_forward", g, opnd, Wf.data_ptr(), None, out.data_ptr(), _lib.cv_epilogue(), s_)
    gin = torch.empty(n, hin, hin, cin, device=dev)
    _lib.call("cv_conv_backward_data", g, gop, Wb.data_ptr(), gin.data_ptr(), _lib.cv_epilogue(), s_)
    wb = _lib.lib().cv_conv_wgrad_workspace_bytes(g, 0)
    work = torch.empty(max(wb // 4, 1), device=dev)
    gw = torch.zeros(wshape, device=dev)
    _lib.call("cv_conv_backward_weight", g, opnd, gop, gw.data_ptr(), None, 0, work.data_ptr(), wb, s_)
    torch.cuda.synchronize()
    return out, gin, gw


@pytest.mark.parametrize("geom", PM_GEOMS, ids=_ids)
def test_pm_matches_image_major(geom, pm_mode):
    from test_gpu_conv_kernels import rel

    set_, L = pm_mode
    a = _run_all(geom, 1, set_)
    assert L.cv_debug_pm_count(1) > 0
    b = _run_all(geom, 0, set_)
    assert L.cv_debug_pm_count(1) == 0
    for name, u, v in zip(("forward", "backward-data", "weight gradient"), a, b):
        assert torch.isfinite(u).all(), name
        assert rel(u, v) < 2e-6, (name, rel(u, v))
