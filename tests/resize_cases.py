"""Resize fixture cases (tests/golden/gen_resize.py -> tests/golden/resize_pil.npz): seeded uint8 images.
Test infrastructure only."""

from __future__ import annotations

import os

import numpy as np

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "resize_pil.npz")

# name, (H, W, C), (out_h, out_w), count, seed
CASES = [
    ("camelyon96", (96, 96, 3), (64, 64), 4, 11),
    ("pacs227", (227, 227, 3), (64, 64), 3, 12),
    ("pacs224", (224, 224, 3), (64, 64), 3, 13),
    ("mnist_identity", (28, 28, 1), (28, 28), 4, 14),
    ("mnist_up64", (28, 28, 1), (64, 64), 2, 15),
    ("rect_50x70", (50, 70, 3), (64, 64), 2, 16),
    ("rect_300x41", (300, 41, 3), (64, 64), 2, 17),
    ("identity64", (64, 64, 3), (64, 64), 2, 18),
    ("odd_33x129", (33, 129, 1), (17, 40), 2, 19),
]


def images(shape, count, seed):
    """Smooth gradients + noise + saturated patches, so results land on rounding boundaries and clamps."""
    H, W, C = shape
    g = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    out = np.empty((count, H, W, C), dtype=np.uint8)
    for i in range(count):
        base = (xx * g.uniform(0.5, 3) + yy * g.uniform(0.5, 3))[:, :, None] + g.uniform(0, 255, (1, 1, C))
        img = np.mod(base + g.normal(0, 20, (H, W, C)), 256)
        img[g.random((H, W)) < 0.05] = 255
        img[g.random((H, W)) < 0.05] = 0
        out[i] = img.astype(np.uint8)
    return out
