"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement of the reference's input transform for the VAE64 datasets and Styled-MNIST:
transforms.Compose([transforms.Resize((64, 64)), transforms.ToTensor()]) on PIL images
(code/run_pacs_downstream_expr.py:88-98, code/run_camelyon17_downstream_expr.ipynb cell 6) and
ToTensor() alone (code/src/utils/data_utils.py:55-73).

The algorithm lives in third-party code absent from /root/reference: torchvision (not installed here;
its PIL path of Resize is Image.resize(size[::-1], BILINEAR)) and Pillow (12.2.0 installed here,
src/libImaging/Resample.c: precompute_coeffs, normalize_coeffs_8bpc, ImagingResampleHorizontal_8bpc /
ImagingResampleVertical_8bpc, ImagingResampleInner).  Restated here:
  * triangle filter, support 1 widened by the downscale factor (antialiasing); per output pixel the
    taps [xmin, xmin + xmax) and weights normalised to sum 1 — all in double, in Pillow's operation order;
  * weights quantised to 22-bit fixed point (round half away from zero);
  * horizontal pass first (int32 accumulation from 1 << 21, >> 22, clamp to [0, 255]), then the
    vertical pass on the 8-bit intermediate;
  * ToTensor: uint8 / 255 in float32.
Pinned to Pillow itself by tests/golden/resize_pil.npz (tests/golden/gen_resize.py runs Image.resize
on seeded images; tests/test_resize_oracle.py checks this restatement bit for bit).
"""

from __future__ import annotations

import math

import numpy as np

PREC = 22


def _filter(x: float) -> float:
    if x < 0.0:
        x = -x
    if x < 1.0:
        return 1.0 - x
    return 0.0


def coeffs(in_size: int, out_size: int):
    """(ksize, bounds [out, 2] = (xmin, taps), fixed-point weights [out, ksize])  (precompute_coeffs +
    normalize_coeffs_8bpc)."""
    in0, in1 = 0.0, float(in_size)
    scale = (in1 - in0) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int64)
    kk = np.zeros((out_size, ksize), dtype=np.int64)
    for xx in range(out_size):
        center = in0 + (xx + 0.5) * scale
        ww = 0.0
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        k = [0.0] * ksize
        for x in range(xmax):
            w = _filter((x + xmin - center + 0.5) * ss)
            k[x] = w
            ww += w
        if ww != 0.0:
            k = [v / ww if i < xmax else v for i, v in enumerate(k)]
        for x in range(ksize):
            v = k[x] * (1 << PREC)
            kk[xx, x] = int(-0.5 + v) if k[x] < 0 else int(0.5 + v)
        bounds[xx] = (xmin, xmax)
    return ksize, bounds, kk


def _pass(img: np.ndarray, bounds, kk, axis: int) -> np.ndarray:
    """One 8bpc pass along `axis` of an int64 [H, W, C] image."""
    src = np.moveaxis(img, axis, 0)
    out = np.empty((len(bounds),) + src.shape[1:], dtype=np.int64)
    for o, (lo, taps) in enumerate(bounds):
        acc = np.full(src.shape[1:], 1 << (PREC - 1), dtype=np.int64)
        for t in range(taps):
            acc += src[lo + t] * kk[o, t]
        out[o] = np.clip(acc >> PREC, 0, 255)
    return np.moveaxis(out, 0, axis)


def resize_u8(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """Image.fromarray(img).resize((out_w, out_h), BILINEAR) for uint8 [H, W] or [H, W, C]."""
    a = np.asarray(img)
    gray = a.ndim == 2
    x = (a[:, :, None] if gray else a).astype(np.int64)
    H, W = x.shape[:2]
    if (H, W) != (out_h, out_w):
        if W != out_w:
            _, bh, kh = coeffs(W, out_w)
            x = _pass(x, bh, kh, 1)
        if H != out_h:
            _, bv, kv = coeffs(H, out_h)
            x = _pass(x, bv, kv, 0)
    x = x.astype(np.uint8)
    return x[:, :, 0] if gray else x


def to_tensor(img_u8: np.ndarray) -> np.ndarray:
    """ToTensor: HWC uint8 -> CHW float32 / 255."""
    a = np.asarray(img_u8)
    if a.ndim == 2:
        a = a[:, :, None]
    return np.ascontiguousarray(a.transpose(2, 0, 1)).astype(np.float32) / np.float32(255)


def transform_batch(images: np.ndarray, index, out_h: int, out_w: int) -> np.ndarray:
    """Resize + ToTensor of images[index] stacked: [n, C, out_h, out_w] float32."""
    return np.stack([to_tensor(resize_u8(images[i], out_h, out_w)) for i in index])
