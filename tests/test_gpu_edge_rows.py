"""Regression for the CV_EDGE_ROWS band-height override of the image-side edge kernels (cv_edge.hip `edge_rows`).

The gather and fused-backward kernels compute ET = 256 pixels per band, one per thread; a band taller than
ET / ws rows (VAE64's 32-wide small grid: more than 8 rows) used to leave the pixels past 256 of its LDS output
tile unwritten, so the epilogue streamed uninitialised LDS into the output and into the BatchNorm sums.  The host
now clamps the override to ET / ws.  The override is read once per process, so the check runs in a child process
with CV_EDGE_ROWS=12 (and =64), on VAE64's conv1 forward and ConvTranspose2d-to-image backward-data (both edge
gathers), against fp64 torch at the kernel bar 1e-5 (tests/test_gpu_conv_kernels.py)."""

import os
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _run_checks():
    from cvhip import _lib
    from test_gpu_conv_kernels import _packed, rel

    dev = torch.device("cuda")
    rng = np.random.default_rng(12)
    s_ = _lib.stream_handle()
    errs = []
    for n, tr, cin, hin, cout, hout, k, s, p in [(8, 0, 3, 64, 32, 32, 4, 2, 1), (8, 1, 32, 32, 3, 64, 4, 2, 1)]:
        g = _lib.cv_conv(n, cin, hin, hin, cout, hout, hout, k, k, s, p, tr)
        wshape = (cin, cout, k, k) if tr else (cout, cin, k, k)
        W = torch.tensor(rng.uniform(-0.2, 0.2, wshape), dtype=torch.float32, device=dev)
        Wf, Wb = _packed(_lib, W, tr)
        if not tr:  # conv1 forward: the edge gather
            x = torch.tensor(rng.standard_normal((n, hin, hin, cin)), dtype=torch.float32, device=dev)
            out = torch.full((n, hout, hout, cout), 7.0, device=dev)
            _lib.call("cv_conv_forward", g, _lib.cv_operand(x.data_ptr(), None, _lib.XF_NONE, 0), Wf.data_ptr(), None,
                      out.data_ptr(), _lib.cv_epilogue(), s_)
            ref = F.conv2d(x.double().cpu().permute(0, 3, 1, 2), W.double().cpu(), stride=s, padding=p)
        else:  # convT5 backward-data: the edge gather over the image-side gradient
            dy = torch.tensor(rng.standard_normal((n, hout, hout, cout)), dtype=torch.float32, device=dev)
            out = torch.full((n, hin, hin, cin), 7.0, device=dev)
            _lib.call("cv_conv_backward_data", g, _lib.cv_operand(dy.data_ptr(), None, _lib.XF_NONE, 0),
                      Wb.data_ptr(), out.data_ptr(), _lib.cv_epilogue(), s_)
            ref = F.conv2d(dy.double().cpu().permute(0, 3, 1, 2), W.double().cpu(), stride=s, padding=p)
        torch.cuda.synchronize()
        errs.append(rel(out, ref.permute(0, 2, 3, 1)))
    return errs


@pytest.mark.parametrize("rows", [12, 64])
def test_edge_rows_override_clamped(rows):
    env = dict(os.environ, CV_EDGE_ROWS=str(rows), PYTHONPATH=os.pathsep.join(
        [HERE, os.path.join(ROOT, "clear-vae_amd"), ROOT, os.environ.get("PYTHONPATH", "")]))
    code = "import test_gpu_edge_rows as t; print('ERRS', *t._run_checks())"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("ERRS")][-1]
    errs = [float(v) for v in line.split()[1:]]
    assert len(errs) == 2 and max(errs) < 1e-5, errs
