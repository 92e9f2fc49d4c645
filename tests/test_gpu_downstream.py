"""`DownstreamMLPTrainer` (reference `code/src/trainer.py:95-165`) with the frozen VAE's
`encode` on the HIP kernels.

The caller pattern is the reference's own (`code/run_styledmnist_downstream_expr.py:100-125`): the trained
VAE is put in eval mode, its parameters are frozen, and an MLP probe (Linear-BN1d-ReLU-Linear) is trained on
mu_c with Adam and cross-entropy, then `evaluate()` returns (AUPR, AUROC) and accuracy.

The oracle side runs `oracle.cpu_ref.encode(train=False)` in fp64 and the same probe in fp64 with torch's Adam.
Tolerances: mu_c within 1e-4 relative (the north_star bar for encoded latents); the probe's parameters after
the steps within 1e-4 relative (the probe itself is plain torch on both sides, so this measures how far the
HIP latents move the probe); the frozen VAE's running statistics must not move in eval mode.
"""

import copy

import numpy as np
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _rel(a, b):
    a = a.detach().double().cpu().reshape(-1)
    b = b.detach().double().cpu().reshape(-1)
    return float((a - b).norm() / (b.norm() + 1e-30))


def _vae(arch, zt, C, sd):
    from src.models.vae import VAE, VAE64

    vae = (VAE if arch == "VAE" else VAE64)(zt, C).cuda()
    vae.load_state_dict({k: torch.as_tensor(np.asarray(v)).float() if np.asarray(v).dtype != np.int64
                         else torch.as_tensor(np.asarray(v)) for k, v in sd.items()})
    return vae


def _probe(d, n_cls):
    torch.manual_seed(7)
    return nn.Sequential(nn.Linear(d, 256), nn.BatchNorm1d(256), nn.ReLU(), nn.Linear(256, n_cls))


@pytest.mark.parametrize("arch,zt,C,n", [("VAE", 16, 1, 128), ("VAE64", 64, 3, 32)])
def test_downstream_probe_matches_oracle(arch, zt, C, n):
    from oracle import cpu_ref as R
    from src.trainer import DownstreamMLPTrainer

    n_cls = 10
    sd = R.det_state(arch, zt, C)
    vae = _vae(arch, zt, C, sd)
    vae.eval()
    for p in vae.parameters():
        p.requires_grad = False
    before = {k: v.clone() for k, v in vae.state_dict().items()}

    batches = []
    for s in range(3):
        x, label, _, _, _ = R.det_inputs(n, C, R.IMAGE[arch], zt, n_cls, seed=11 + s)
        batches.append((torch.tensor(x, dtype=torch.float32), torch.tensor(label).reshape(-1, 1)))

    probe0 = _probe(zt // 2, n_cls)
    mlp = copy.deepcopy(probe0).cuda()
    opt = torch.optim.Adam(mlp.parameters(), lr=3e-4)
    tr = DownstreamMLPTrainer(vae, mlp, opt, nn.CrossEntropyLoss(), 10, torch.device("cuda"))
    tr._train(batches, verbose=False, epoch_id=0)

    # oracle: fp64 eval-mode encode, fp64 probe, torch Adam
    P = R.to_torch(sd, requires_grad=False)
    omlp = copy.deepcopy(probe0).double()
    oopt = torch.optim.Adam(omlp.parameters(), lr=3e-4)
    omlp.train()
    for X, y in batches:
        mu_c = R.encode(P, X.double(), arch, train=False)[0]
        with torch.no_grad():
            got = vae.encode(X.cuda())[0]
        assert _rel(got, mu_c) < TOL
        oopt.zero_grad()
        loss = nn.functional.cross_entropy(omlp(mu_c), y.reshape(-1).long())
        loss.backward()
        oopt.step()

    for (k, a), (_, b) in zip(mlp.state_dict().items(), omlp.state_dict().items()):
        if k == "0.bias":
            # this bias feeds a train-mode BatchNorm1d: its gradient is mathematically zero, and Adam
            # normalises the rounding noise on either side into a step of up to lr per update
            assert float((a.double().cpu() - probe0.state_dict()[k].double()).abs().max()) <= 3 * 3e-4 * 1.01
        elif k == "1.running_mean":
            # running_mean = sum_t 0.1 * 0.9^(2-t) * mean_n(W_t mu + b_t): it carries the 0.bias noise above,
            # |b_t - b_0| <= t * lr on either side, so per element the two sides may differ by up to
            # 0.1 * (0.9 * 1 + 1 * 2) * lr from the bias alone (running_var is shift-invariant: no such term)
            bias_drift = 0.1 * (0.9 * 1 + 1.0 * 2) * 3e-4 * 1.01
            diff = (a.double().cpu() - b.double()).abs()
            assert float(diff.max()) <= bias_drift + TOL * float(b.abs().max()), k
        elif a.dtype.is_floating_point:
            assert _rel(a, b) < TOL, k
    # eval-mode BatchNorm in the frozen VAE: nothing moved, no gradients were made
    for k, v in vae.state_dict().items():
        assert torch.equal(v, before[k]), k
    assert all(p.grad is None for p in vae.parameters())

    (aupr, auroc), acc = tr.evaluate(batches, verbose=False, epoch_id=0)
    omlp.eval()
    with torch.no_grad():
        ologits = torch.cat([omlp(R.encode(P, X.double(), arch, train=False)[0]) for X, _ in batches])
    oy = torch.cat([y.reshape(-1) for _, y in batches])
    oacc = float((ologits.argmax(1) == oy).double().mean())
    assert abs(float(acc) - oacc) <= 1.0 / len(oy) + 1e-12
    assert set(aupr) == set(auroc) == set(range(int(oy.max()) + 1))
