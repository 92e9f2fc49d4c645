"""Device-resident datasets and loaders: the producer side of the training step.

The reference builds batches on the host: StyledMNIST keeps a materialised list of PIL images and applies
ToTensor per item (code/src/utils/data_utils.py:55-77); PACS and Camelyon17 resize every PIL image with
transforms.Resize((64, 64)) + ToTensor() in the DataLoader (code/run_pacs_downstream_expr.py:88-98,
code/run_camelyon17_downstream_expr.ipynb cell 6).  DeviceImageDataset holds the raw uint8 images in HBM
(Camelyon17's 302k 96x96x3 training patches are 8.3 GB: the whole set fits on one MI355X many times over)
and DeviceLoader yields (X, label[, style]) batches made by one cv_load_batch_u8 launch each — the same
values as the reference's transforms, bit for bit (tests/test_gpu_data.py).  The style corruptions that
generate Styled-MNIST (corruption_utils: skimage / wand / cv2) stay a host-side, once-per-dataset step
and are outside the hot path: DeviceImageDataset takes their uint8 output.
"""

from __future__ import annotations

import numpy as np
import torch

from cvhip.data import load_batch


class DeviceImageDataset:
    """uint8 images [N, H, W] or [N, H, W, C] + int labels (+ style labels) on the device; items come out
    as transforms.Compose([Resize(size), ToTensor()]) would make them (size=None: ToTensor only)."""

    def __init__(self, images, labels, styles=None, size=None, device="cuda") -> None:
        imgs = torch.as_tensor(np.asarray(images) if not isinstance(images, torch.Tensor) else images)
        if imgs.dtype != torch.uint8 or imgs.dim() not in (3, 4):
            raise ValueError("images: uint8 [N, H, W] or [N, H, W, C]")
        self.images = imgs.to(device).contiguous()
        self.labels = torch.as_tensor(labels).reshape(-1).to(device=device, dtype=torch.int64)
        self.styles = None if styles is None else torch.as_tensor(styles).reshape(-1).to(device=device,
                                                                                         dtype=torch.int64)
        if self.labels.numel() != self.images.shape[0]:
            raise ValueError("one label per image")
        if self.styles is not None and self.styles.numel() != self.images.shape[0]:
            raise ValueError("one style label per image")
        H, W = self.images.shape[1:3]
        self.size = tuple(size) if size is not None else (H, W)

    @classmethod
    def from_items(cls, items, size=None, device="cuda"):
        """From (image, label[, style]) items, e.g. a materialised StyledMNIST list (data_utils.py:61-65):
        images are PIL images or uint8 arrays of one size; uploaded once."""
        imgs, labels, styles = [], [], []
        for it in items:
            imgs.append(np.asarray(it[0], dtype=np.uint8))
            labels.append(int(it[1]))
            if len(it) > 2:
                styles.append(int(it[2]))
        return cls(np.stack(imgs), labels, styles if styles else None, size, device)

    def __len__(self) -> int:
        return self.images.shape[0]

    def __getitem__(self, idx) -> tuple:
        k, n = int(idx), len(self)
        if not -n <= k < n:  # (list indexing semantics, like the reference's materialised list)
            raise IndexError(f"index {k} out of range for {n} images")
        i = torch.tensor([k % n], device=self.images.device)
        x, y, s = load_batch(self.images, i, self.size, self.labels, self.styles, checked=False)
        return (x[0], y[0]) if s is None else (x[0], y[0], s[0])

    def batch(self, index: torch.Tensor, out: torch.Tensor | None = None, checked: bool = True) -> tuple:
        x, y, s = load_batch(self.images, index, self.size, self.labels, self.styles, out=out, checked=checked)
        return (x, y) if s is None else (x, y, s)


class DeviceLoader:
    """torch DataLoader semantics over a DeviceImageDataset (batch_size, shuffle, drop_last); the
    permutation is drawn on the device, batches are (X, label[, style]) device tensors."""

    def __init__(self, dataset: DeviceImageDataset, batch_size: int = 1, shuffle: bool = False,
                 drop_last: bool = False, generator: torch.Generator | None = None) -> None:
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.generator = generator

    def __len__(self) -> int:
        n = len(self.dataset)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        n = len(self.dataset)
        dev = self.dataset.images.device
        if self.shuffle:
            order = torch.randperm(n, device=dev, generator=self.generator)
        else:
            order = torch.arange(n, device=dev)
        for b in range(len(self)):
            yield self.dataset.batch(order[b * self.batch_size:(b + 1) * self.batch_size], checked=False)
