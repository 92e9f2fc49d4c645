"""The register-resident NT-Xent variants (csrc/cv_ntxent.hpp ntxent_*_reg_body: cosine similarity, n <= 512 with
d <= 8 or n <= 256 with d <= 32, in 16-byte rows — MNIST's bs = 512, z = 16; VAE64's bs <= 256, z = 64) against the LDS-staged kernels they replace (cv_debug_nt_reg(0)).
Reference: losses.py:98-137 (contrastive_loss / snn_loss through the cosine similarity, losses.py:70-76).

Both variants do the same arithmetic in the same order, so the row log-sum-exps, the losses and the gradients must be
BIT-identical: batches at, below and not a multiple of the tile (512, 300, 64, 5), d = 8 and 4, the two positive-set
rules (ps = 1: different label, ps = 0: same label), accumulate on and off, the heads' strided layout (ld = 4d), a
zero row (the clamped-norm path of the gradient) and rows without positives (non-finite rows, dropped from the
mean); VAE64's d = 32 at n = 256 / 128 and d = 16.  The fused step through the reg path is held to the fp64 oracle by test_gpu_aux.py / test_gpu_parity.py."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(reg, mu_all, lab, n, d, ps, accumulate, ld, seed_grad):
    from cvhip import _lib

    L = _lib.lib()
    prev = L.cv_debug_nt_reg(1 if reg else 0)
    try:
        dev = mu_all.device
        lse = torch.full((2 * n,), 7.0, dtype=torch.float32, device=dev)
        loss = torch.zeros((), dtype=torch.float32, device=dev)
        dmu = seed_grad.clone()
        dlv = seed_grad.clone() * 0.5
        gsc = torch.tensor([0.75], dtype=torch.float32, device=dev)
        br = _lib.cv_ntxent_branch(mu_all.data_ptr(), None, ld, ps, dmu.data_ptr(), dlv.data_ptr(), ld,
                                   gsc.data_ptr(), 1.25, loss.data_ptr(), lse.data_ptr())
        _lib.call("cv_ntxent", br, 1, lab.data_ptr(), n, d, _lib.SIM["cosine"], 0.1, 2, accumulate,
                  _lib.stream_handle())
        torch.cuda.synchronize()
    finally:
        L.cv_debug_nt_reg(prev)
    return lse.cpu(), loss.cpu(), dmu.cpu(), dlv.cpu()


@pytest.mark.parametrize("n,d", [(512, 8), (300, 8), (64, 8), (5, 8), (512, 4), (64, 4), (256, 32), (128, 32),
                                 (100, 16), (7, 32)])
@pytest.mark.parametrize("ps", [1, 0])
@pytest.mark.parametrize("accumulate", [0, 1])
def test_reg_variant_bit_identical(n, d, ps, accumulate):
    rng = np.random.default_rng(1000 * n + 10 * d + 2 * ps + accumulate)
    dev = torch.device("cuda")
    ld = 4 * d  # (the heads block: rows of [mu_c, lv_c, mu_s, lv_s])
    mu_all = torch.tensor(rng.standard_normal((n, ld)), dtype=torch.float32, device=dev)
    mu_all[min(3, n - 1), :d] = 0.0  # a zero row: clamped norm
    lab_np = rng.integers(0, 10, n)
    lab_np[0] = 99  # unique label: no positives under ps = 0 (a non-finite row)
    lab = torch.tensor(lab_np, dtype=torch.int64, device=dev)
    seed_grad = torch.tensor(rng.standard_normal((n, ld)), dtype=torch.float32, device=dev)
    a = _run(True, mu_all, lab, n, d, ps, accumulate, ld, seed_grad)
    b = _run(False, mu_all, lab, n, d, ps, accumulate, ld, seed_grad)
    for x, y, name in zip(a, b, ("lse", "loss", "dmu", "dlv")):
        assert torch.equal(x.view(torch.int32), y.view(torch.int32)), (name, (x - y).abs().max())
    if n >= 64:  # (at n = 5 every row may lack positives: the mean over no finite row is NaN in both)
        assert torch.isfinite(a[1]), a[1]


def test_reg_variant_is_taken():
    """The variant is the default for the MNIST shape and the switch really changes the launched kernel."""
    import ctypes

    from cvhip import _lib

    L = _lib.lib()
    dev = torch.device("cuda")
    n, d = 512, 8
    mu_all = torch.randn(n, 4 * d, device=dev)
    lab = torch.randint(0, 10, (n,), device=dev)
    seed = torch.zeros(n, 4 * d, device=dev)
    names = {}
    for reg in (1, 0):
        prev = L.cv_debug_kernel_log(1)
        try:
            _run(bool(reg), mu_all, lab, n, d, 1, 0, 4 * d, seed)
            buf = ctypes.create_string_buffer(1 << 16)
            k = L.cv_debug_kernel_names(buf, len(buf))
        finally:
            L.cv_debug_kernel_log(prev)
        names[reg] = buf.value.decode().split("\n") if k else []
    assert L.cv_debug_nt_reg(-1) == 1
    assert sum("reg_kernel" in k for k in names[1]) == 2, names[1]
    assert not any("reg_kernel" in k for k in names[0]), names[0]
