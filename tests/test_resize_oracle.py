"""The input-transform oracle (oracle/resize_ref.py) pinned to Pillow (tests/golden/resize_pil.npz, made by
tests/golden/gen_resize.py with Image.resize(BILINEAR) — the operation behind the reference's
transforms.Resize((64, 64)) on PIL images), and the C-ABI's host-side plan builder (cv_resize_plan in
libclearvae_hip.so) checked against the oracle's coefficients, and a CPU emulation of the kernel's tiling
of that plan.  Bit-exact throughout.  CPU only (the plan builder is host code)."""

import ctypes

import numpy as np
import pytest

from oracle import resize_ref as RR
from resize_cases import CASES, FIXTURE, images


@pytest.fixture(scope="module")
def fixture():
    with np.load(FIXTURE, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_oracle_matches_pillow(fixture, case):
    name, shape, (oh, ow), count, seed = case
    imgs = images(shape, count, seed)
    ck = np.array([imgs.astype(np.int64).sum(), (imgs.astype(np.int64) ** 2).sum()])
    assert np.array_equal(ck, fixture[name + "__checksum"]), "image generator drifted"
    ref = fixture[name + "__out"]
    for i in range(count):
        got = RR.resize_u8(imgs[i] if shape[2] > 1 else imgs[i, :, :, 0], oh, ow)
        got = got if got.ndim == 3 else got[:, :, None]
        assert np.array_equal(got, ref[i]), (name, i, int(np.abs(got.astype(int) - ref[i]).max()))


def _plan(in_h, in_w, out_h, out_w):
    from cvhip import _lib

    L = _lib.lib()
    words = int(L.cv_resize_plan_words(in_h, in_w, out_h, out_w))
    buf = (ctypes.c_int32 * words)()
    _lib.call("cv_resize_plan", in_h, in_w, out_h, out_w, ctypes.addressof(buf), words)
    return np.frombuffer(buf, dtype=np.int32).copy()


SIZES = [(96, 96, 64, 64), (227, 227, 64, 64), (224, 224, 64, 64), (28, 28, 28, 28), (28, 28, 64, 64),
         (50, 70, 64, 64), (300, 41, 64, 64), (33, 129, 17, 40), (1000, 999, 64, 64), (5, 7, 64, 64)]


@pytest.mark.parametrize("sz", SIZES, ids=["x".join(map(str, s)) for s in SIZES])
def test_plan_matches_oracle(sz):
    in_h, in_w, out_h, out_w = sz
    P = _plan(*sz)
    kh, kv, ybf = int(P[0]), int(P[1]), int(P[2])
    o = 16
    bh = P[o:o + 2 * out_w].reshape(out_w, 2)
    o += 2 * out_w
    kkh = P[o:o + out_w * kh].reshape(out_w, kh)
    o += out_w * kh
    bv = P[o:o + 2 * out_h].reshape(out_h, 2)
    o += 2 * out_h
    kkv = P[o:o + out_h * kv].reshape(out_h, kv)
    k1, b1, c1 = RR.coeffs(in_w, out_w)
    k2, b2, c2 = RR.coeffs(in_h, out_h)
    assert (kh, kv) == (k1, k2)
    assert np.array_equal(bh, b1) and np.array_equal(kkh, c1)
    assert ybf == b2[0, 0]
    assert np.array_equal(bv[:, 0] + ybf, b2[:, 0]) and np.array_equal(bv[:, 1], b2[:, 1])
    assert np.array_equal(kkv, c2)


def _emulate(img, P, out_h, out_w, ty):
    """The kernel's arithmetic on the C plan, tile by tile (cv_data.hip load_batch_kernel), on the CPU."""
    H, W, C = img.shape
    kh, kv, ybf = int(P[0]), int(P[1]), int(P[2])
    o = 16
    bh = P[o:o + 2 * out_w].reshape(out_w, 2)
    o += 2 * out_w
    kkh = P[o:o + out_w * kh].reshape(out_w, kh).astype(np.int64)
    o += out_w * kh
    bv = P[o:o + 2 * out_h].reshape(out_h, 2)
    o += 2 * out_h
    kkv = P[o:o + out_h * kv].reshape(out_h, kv).astype(np.int64)
    out = np.zeros((C, out_h, out_w), dtype=np.float32)
    src = img.astype(np.int64)
    for y0 in range(0, out_h, ty):
        y1 = min(out_h, y0 + ty)
        r0, r1 = bv[y0, 0], bv[y1 - 1, 0] + bv[y1 - 1, 1]
        tmp = np.zeros((r1 - r0, out_w, C), dtype=np.int64)
        for xx in range(out_w):
            acc = np.full((r1 - r0, C), 1 << 21, dtype=np.int64)
            for t in range(bh[xx, 1]):
                acc += src[ybf + r0:ybf + r1, bh[xx, 0] + t, :] * kkh[xx, t]
            tmp[:, xx, :] = np.clip(acc >> 22, 0, 255)
        for yy in range(y0, y1):
            acc = np.full((out_w, C), 1 << 21, dtype=np.int64)
            for t in range(bv[yy, 1]):
                acc += tmp[bv[yy, 0] - r0 + t] * kkv[yy, t]
            out[:, yy, :] = (np.clip(acc >> 22, 0, 255).astype(np.float32) / np.float32(255)).T
    return out


@pytest.mark.parametrize("case", CASES[:3] + CASES[5:7], ids=[c[0] for c in CASES[:3] + CASES[5:7]])
@pytest.mark.parametrize("ty", [16, 5])
def test_kernel_tiling_emulation(fixture, case, ty):
    name, shape, (oh, ow), count, seed = case
    img = images(shape, 1, seed)[0]
    P = _plan(shape[0], shape[1], oh, ow)
    got = _emulate(img, P, oh, ow, ty)
    ref = fixture[name + "__out"][0].transpose(2, 0, 1).astype(np.float32) / np.float32(255)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("sz", SIZES, ids=["x".join(map(str, s)) for s in SIZES])
def test_resize_plan_tiles(sz):
    """cvhip.data.ResizePlan (host side): tiles fit the LDS budget, small batches get shorter tiles."""
    from cvhip.data import ResizePlan

    in_h, in_w, out_h, out_w = sz
    p = ResizePlan(in_h, in_w, out_h, out_w, 3, "cpu")
    words = p.plan.numel()
    for ty, tr in p.tiles:
        assert 4 * (words - 16) + 16 + tr * (out_w + (in_w if p.stage else 0)) * 3 <= 64 * 1024
    ty_big, _ = p.tile_for(4096)
    ty_small, _ = p.tile_for(8)
    assert ty_big >= ty_small
