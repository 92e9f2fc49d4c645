"""Device-side input pipeline: Resize + ToTensor of uint8 images resident in HBM.

The reference prepares every batch on the host — torchvision Resize((64, 64)) + ToTensor() per PIL
image in the DataLoader workers (code/run_pacs_downstream_expr.py:88-98,
code/run_camelyon17_downstream_expr.ipynb cell 6; Styled-MNIST: ToTensor over a materialised list,
code/src/utils/data_utils.py:55-73) — and its L4 runs were loader-bound.  Here the raw
uint8 images stay on the device and one cv_load_batch_u8 launch per batch gathers the sampled images,
resamples them with Pillow's exact integer arithmetic, converts to fp32 NCHW / 255 and gathers the
labels.  Bit-exact with Pillow + ToTensor (tests/test_resize_oracle.py, tests/test_gpu_data.py).
"""

from __future__ import annotations

import ctypes

import torch

from . import _lib

_LDS = 48 * 1024  # tile rows staged per workgroup


class ResizePlan:
    """Pillow's resampling coefficients for one (in_h, in_w) -> (out_h, out_w), on the device."""

    _cache: dict = {}

    def __init__(self, in_h: int, in_w: int, out_h: int, out_w: int, c: int, device):
        L = _lib.lib()
        self.out_h = out_h
        words = int(L.cv_resize_plan_words(in_h, in_w, out_h, out_w))
        host = (ctypes.c_int32 * words)()
        _lib.call("cv_resize_plan", in_h, in_w, out_h, out_w, ctypes.addressof(host), words)
        # output rows per workgroup: enough workgroups per image for small batches; the tile's source rows
        # staged in LDS (coalesced loads) when they fit, else read from global memory in the horizontal pass
        def rows(ty):
            return int(L.cv_resize_tile_rows(ctypes.addressof(host), ty))

        body = 4 * (words - 16) + 16  # the plan's bounds and coefficients, staged in LDS too

        def fits(ty, stage):
            return body + rows(ty) * (out_w + (in_w if stage else 0)) * c + 16 <= _LDS

        self.stage = 1
        ty = min(out_h, 16)
        while ty > 1 and not fits(ty, 1):
            ty //= 2
        if not fits(ty, 1):
            self.stage = 0
            ty = min(out_h, 16)
            while ty > 1 and not fits(ty, 0):
                ty //= 2
            if not fits(ty, 0):
                raise ValueError(f"resize {in_h}x{in_w} -> {out_h}x{out_w}: downscale too large for one tile")
        # (ty, tile rows) from the largest tile down: small batches take shorter tiles so the launch still
        # has ~2048 workgroups (8 per CU) in flight
        self.tiles = []
        t = ty
        while t >= 1:
            self.tiles.append((t, rows(t)))
            t //= 2
        self.ty, self.tile_rows = self.tiles[0]
        self.plan = torch.tensor(list(host), dtype=torch.int32).to(device)
        self.shape = (in_h, in_w, out_h, out_w, c)

    def tile_for(self, n: int):
        out_h = self.out_h
        for ty, tr in self.tiles:
            if n * (-(-out_h // ty)) >= 2048:
                return ty, tr
        return self.tiles[-1] if len(self.tiles) < 3 else self.tiles[2]

    @classmethod
    def get(cls, in_h, in_w, out_h, out_w, c, device):
        key = (in_h, in_w, out_h, out_w, c, str(device))
        p = cls._cache.get(key)
        if p is None:
            p = cls._cache[key] = cls(in_h, in_w, out_h, out_w, c, device)
        return p


def load_batch(images: torch.Tensor, index: torch.Tensor | None, out_hw, labels=None, styles=None, out=None,
               stream=None, checked: bool = True):
    """Resize + ToTensor of images[index] (uint8 [N, H, W] or [N, H, W, C] on the device) into fp32
    [n, C, out_h, out_w]; returns (X, labels[index] or None, styles[index] or None).

    The kernel addresses images / labels / styles through `index` without bounds checks, so a caller's
    index is range-checked on the host first (IndexError, as tensor indexing would raise; one device
    read).  checked=False skips that for indices the caller made in range itself (DeviceLoader's own
    permutation)."""
    if images.device.type != "cuda" or images.dtype != torch.uint8:
        raise RuntimeError("clear-vae_amd: load_batch needs a uint8 image tensor on the ROCm device")
    imgs = images if images.dim() == 4 else images.unsqueeze(-1)
    if not imgs.is_contiguous():
        raise ValueError("images must be contiguous HWC")
    N, H, W, C = imgs.shape
    oh, ow = out_hw
    idx = None
    n = N
    if index is not None:
        idx = index.to(device=images.device, dtype=torch.int64).contiguous()
        n = idx.numel()
        if checked and n:
            lo, hi = (int(v) for v in torch.aminmax(idx))
            if lo < 0 or hi >= N:
                raise IndexError(f"load_batch: index out of range [{lo}, {hi}] for {N} images")
    plan = ResizePlan.get(H, W, oh, ow, C, images.device)
    if out is None:
        out = torch.empty(n, C, oh, ow, dtype=torch.float32, device=images.device)
    assert out.shape == (n, C, oh, ow) and out.is_contiguous() and out.dtype == torch.float32
    lab_out = sty_out = None
    if labels is not None:
        labels = labels.to(device=images.device, dtype=torch.int64).contiguous()
        lab_out = torch.empty(n, dtype=torch.int64, device=images.device)
    if styles is not None:
        styles = styles.to(device=images.device, dtype=torch.int64).contiguous()
        sty_out = torch.empty(n, dtype=torch.int64, device=images.device)
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    ty, tile_rows = plan.tile_for(n)
    _lib.call("cv_load_batch_u8", imgs.data_ptr(), H, W, C, ptr(idx), n, plan.plan.data_ptr(), oh, ow, ty,
              tile_rows, plan.stage, out.data_ptr(), ptr(labels), ptr(lab_out), ptr(styles), ptr(sty_out),
              _lib.stream_handle() if stream is None else stream)
    return out, lab_out, sty_out
