"""Golden vectors of the reference's contrastive_loss with its supcon loss names (development container only).

Imports the REAL reference (read-only, /root/reference/code, never copied) and evaluates
src.losses.contrastive_loss(mu, logvar, label, sim_fn, tau, loss_name=...) (losses.py:98-126, with
supcon_in_loss / supcon_out_loss at :140-170) in fp64 on seeded inputs, for every similarity and both ps
settings.  Writes tests/golden/supcon.npz (inputs + the scalar per case).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_supcon.py
"""

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference/code")

from src.losses import contrastive_loss  # noqa: E402  (the reference's)

SIMS = ("cosine", "l2", "jeffrey", "mahalanobis", "modified_l2")


def main():
    rng = np.random.default_rng(17)
    n, d = 48, 8
    mu = rng.standard_normal((n, d))
    lv = rng.standard_normal((n, d)) * 0.3
    label = rng.integers(0, 5, size=n).astype(np.int64)
    out = {"mu": mu, "logvar": lv, "label": label, "tau": np.array(0.5)}
    for loss in ("supcon_in_loss", "supcon_out_loss"):
        for sim in SIMS:
            for ps in (False, True):
                v = contrastive_loss(torch.tensor(mu), torch.tensor(lv), torch.tensor(label), sim, 0.5,
                                     loss_name=loss, ps=ps)
                out[f"{loss}__{sim}__ps{int(ps)}"] = np.array(float(v))
    np.savez(os.path.join(HERE, "supcon.npz"), **out)
    print("wrote", len(out) - 4, "cases")


if __name__ == "__main__":
    main()
