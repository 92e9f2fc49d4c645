"""The device input pipeline (cv_load_batch_u8 via cvhip.data / src.utils.data_utils)
against Pillow + ToTensor: bit-exact on the Pillow fixtures (tests/golden/resize_pil.npz) and against the
oracle (oracle/resize_ref.py, pinned to those fixtures) at the configurations' full batch sizes
(Camelyon17 96x96 -> 64x64 at bs 1024, PACS 227x227 -> 64x64 at bs 128, Styled-MNIST ToTensor at
bs 512), plus size-independent properties over the whole batch (gather = index of the full load;
label / style gather) and the loader's epoch semantics."""

import numpy as np
import pytest
import torch

from oracle import resize_ref as RR
from resize_cases import CASES, FIXTURE, images

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fixture():
    with np.load(FIXTURE, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_load_batch_matches_pillow(fixture, case):
    from cvhip.data import load_batch

    name, shape, (oh, ow), count, seed = case
    imgs = images(shape, count, seed)
    dev = torch.tensor(imgs if shape[2] > 1 else imgs[:, :, :, 0], device="cuda")
    idx = torch.arange(count - 1, -1, -1, device="cuda")  # reversed: exercises the gather
    lab = torch.arange(100, 100 + count, device="cuda")
    x, y, s = load_batch(dev, idx, (oh, ow), labels=lab, styles=lab * 2)
    ref = fixture[name + "__out"][::-1].transpose(0, 3, 1, 2).astype(np.float32) / np.float32(255)
    got = x.cpu().numpy()
    assert np.array_equal(got, ref), (name, float(np.abs(got - ref).max()))
    assert torch.equal(y.cpu(), torch.arange(100 + count - 1, 99, -1))
    assert torch.equal(s.cpu(), 2 * torch.arange(100 + count - 1, 99, -1))


@pytest.mark.parametrize("shape,out,n,N", [((96, 96, 3), (64, 64), 1024, 1500), ((227, 227, 3), (64, 64), 128, 200),
                                          ((28, 28, 1), (28, 28), 512, 700)],
                         ids=["camelyon96_bs1024", "pacs227_bs128", "mnist_bs512"])
def test_full_batch(shape, out, n, N):
    from cvhip.data import load_batch

    g = np.random.default_rng(5)
    imgs = g.integers(0, 256, size=(N,) + shape, dtype=np.uint8)
    dev = torch.tensor(imgs, device="cuda")
    idx_np = g.integers(0, N, size=n)  # with repeats
    x, _, _ = load_batch(dev, torch.tensor(idx_np, device="cuda"), out)
    full, _, _ = load_batch(dev, None, out)
    # size-independent: the gathered batch is the full load indexed (every row, bit for bit)
    assert torch.equal(x, full[torch.tensor(idx_np, device="cuda")])
    # oracle on a sample of the rows
    xs = x.cpu().numpy()
    for r in g.choice(n, 12, replace=False):
        ref = RR.to_tensor(RR.resize_u8(imgs[idx_np[r]] if shape[2] > 1 else imgs[idx_np[r], :, :, 0], *out))
        assert np.array_equal(xs[r], ref), r


def test_device_loader_epoch():
    from src.utils.data_utils import DeviceImageDataset, DeviceLoader

    g = np.random.default_rng(7)
    N = 1000
    imgs = g.integers(0, 256, size=(N, 96, 96, 3), dtype=np.uint8)
    labels = g.integers(0, 2, size=N)
    styles = g.integers(0, 5, size=N)
    ds = DeviceImageDataset(imgs, labels, styles, size=(64, 64))
    dl = DeviceLoader(ds, batch_size=128, shuffle=True, generator=torch.Generator(device="cuda").manual_seed(0))
    assert len(dl) == 8
    seen_l, seen_s, count = [], [], 0
    for X, y, s in dl:
        assert X.shape[1:] == (3, 64, 64) and X.dtype == torch.float32 and X.device.type == "cuda"
        seen_l.append(y)
        seen_s.append(s)
        count += X.shape[0]
    assert count == N
    assert sorted(torch.cat(seen_l).tolist()) == sorted(labels.tolist())
    assert sorted(torch.cat(seen_s).tolist()) == sorted(styles.tolist())
    assert len(DeviceLoader(ds, 128, drop_last=True)) == 7
    x0, y0, s0 = ds[3]
    assert np.array_equal(x0.cpu().numpy(), RR.to_tensor(RR.resize_u8(imgs[3], 64, 64)))
    assert int(y0) == labels[3] and int(s0) == styles[3]


def test_train_from_device_loader():
    """CLEAR-VAE (VAE64) trained from raw 96x96 uint8 images resident in HBM: the loader feeds the fused
    step with no host round trip."""
    from src.utils.data_utils import DeviceImageDataset, DeviceLoader
    from src.utils.trainer_utils import get_clearvae_trainer

    torch.manual_seed(0)
    g = np.random.default_rng(8)
    imgs = g.integers(0, 256, size=(256, 96, 96, 3), dtype=np.uint8)
    ds = DeviceImageDataset(imgs, g.integers(0, 2, size=256), g.integers(0, 3, size=256), size=(64, 64))
    dl = DeviceLoader(ds, batch_size=64, shuffle=True)
    tr = get_clearvae_trainer(beta=1 / 32, ps=True, vae_lr=1e-4, z_dim=64, alpha=100, temperature=0.1,
                              device="cuda", vae_arch="VAE64", in_channel=3, verbose_period=100)
    tr.fit(2, dl)
    assert tr._engine is not None, "fused engine not used"
    assert torch.isfinite(tr._engine.last_workspace(64).losses[:5]).all()
