"""Test helper (no tests here): the ReLU activity pattern a fused HIP step chose, for the mask-pinned gradient
checks (tests/test_gpu_maskpinned.py, tests/test_gpu_bf16.py, tests/test_gpu_dp.py via tests/dp_gpu_worker.py).

Device masks: the forward stores pre-BN activations (NHWC); the mask of layer l is BN_l(y_l) > 0 evaluated by
cv_bn_apply with the step's own batch statistics and the step's (pre-update) BN affine parameters — the arithmetic
of the GEMM prologues' BN+ReLU transform (bn_out in cv_common.hpp, fmaf((x - mu), sc, beta)); the BatchNorm1d's
mask is its stored output ah > 0.  Call it after the backward and before Adam moves gamma / beta
(ClearStep.step(..., before_update=...)).  The masks feed oracle/cpu_ref.py `masks=`."""

import torch


def device_masks(eng, ws, n):
    from cvhip import _lib

    sp = eng.spec
    s = _lib.stream_handle()
    masks = {}
    for li, c in enumerate(sp.enc):
        y = ws.y_enc[li]
        out = torch.empty_like(y)
        _lib.call("cv_bn_apply", ws.bn_enc[li].cv(True), y.data_ptr(), out.data_ptr(), n * c.h_out * c.w_out,
                  c.c_out, 1, c.c_out, 0, s)
        masks[f"encoder.{3 * li + 2}"] = (out > 0).view(n, c.h_out, c.w_out, c.c_out).permute(0, 3, 1, 2)
    Cu, Hu, Wu = sp.unflat
    masks["decoder.2"] = (ws.ah > 0).view(n, Hu * Wu, Cu).permute(0, 2, 1).reshape(n, Cu * Hu * Wu)
    for li, c in enumerate(sp.dec[:-1]):
        y = ws.y_dec[li]
        out = torch.empty_like(y)
        _lib.call("cv_bn_apply", ws.bn_dec[li].cv(True), y.data_ptr(), out.data_ptr(), n * c.h_out * c.w_out,
                  c.c_out, 1, c.c_out, 0, s)
        masks[f"decoder.{4 + 3 * li + 2}"] = (out > 0).view(n, c.h_out, c.w_out, c.c_out).permute(0, 3, 1, 2)
    torch.cuda.synchronize()
    return {k: v.double().cpu() for k, v in masks.items()}


def masks_to_numpy(masks):
    """bool arrays (compact for a process queue)"""
    return {k: v.numpy() > 0.5 for k, v in masks.items()}


def masks_from_numpy(masks):
    return {k: torch.tensor(v, dtype=torch.float64) for k, v in masks.items()}
