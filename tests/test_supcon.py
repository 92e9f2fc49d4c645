"""contrastive_loss with the reference's supcon loss names (src/losses.py:98-126 dispatching through
eval(loss_name) to supcon_in_loss / supcon_out_loss, :140-170).  These losses are off the trained path
(no trainer, factory or script passes them), so the mirror evaluates the reference's own torch
composition; held bit-for-bit-close (1e-12, fp64) to golden values the real reference produced
(tests/golden/gen_supcon.py).  An unknown loss name raises NameError as the reference's eval does."""

import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _fx():
    with np.load(os.path.join(HERE, "golden", "supcon.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("loss", ["supcon_in_loss", "supcon_out_loss"])
@pytest.mark.parametrize("sim", ["cosine", "l2", "jeffrey", "mahalanobis", "modified_l2"])
@pytest.mark.parametrize("ps", [False, True])
def test_supcon_matches_reference(loss, sim, ps):
    from src.losses import contrastive_loss

    fx = _fx()
    v = contrastive_loss(torch.tensor(fx["mu"]), torch.tensor(fx["logvar"]), torch.tensor(fx["label"]), sim,
                         float(fx["tau"]), loss_name=loss, ps=ps)
    ref = float(fx[f"{loss}__{sim}__ps{int(ps)}"])
    assert abs(float(v) - ref) <= 1e-12 * max(abs(ref), 1.0), (float(v), ref)


def test_unknown_loss_name_raises_like_eval():
    from src.losses import contrastive_loss

    fx = _fx()
    with pytest.raises(NameError):
        contrastive_loss(torch.tensor(fx["mu"]), torch.tensor(fx["logvar"]), torch.tensor(fx["label"]), "cosine",
                         0.5, loss_name="no_such_loss")
