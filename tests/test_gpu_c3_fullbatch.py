"""configs[2] at its own batch: one fused VAE64 CLEAR-MIM CLUB-S step (CelebA 64x64, z = 64, 3 channels, n = 256 —
the bench's `c3` key) against the fp64 oracle (oracle/cpu_ref.py mim_step, pinned to the real reference by
tests/golden), on identical deterministic weights, inputs, noise and permutation.

Reference step: /root/reference/code/src/trainer.py:820-897 (ClearMIMVAETrainer._train: the VAE step :848-869 with
the CLUB-S penalty of src/models/mi_estimator.py:108-131, then 5 estimator updates :873-888).

Checked:
  * rec, kl_c, kl_s, c_loss within 1e-4 relative (north_star's bar), the signed MI term within 1e-4 * max(|mi|, 1);
  * every VAE gradient tensor against the oracle run with the ReLU masks the device chose (tests/maskpin.py,
    the mask-pinned bars of tests/test_gpu_maskpinned.py: median < 5e-6, every tensor < max(1e-5, 8x its fp32
    floor));
  * the 5 estimator learning losses against the oracle's estimator updated by torch Adam after the VAE's torch
    Adam step (1e-4 relative, as tests/test_gpu_parity.py::test_fused_mim_step)."""

import numpy as np
import pytest
import torch

from maskpin import device_masks
from test_gpu_maskpinned import FLOOR_X, MEDIAN_TOL, WORST_TOL
from test_gpu_parity import LOSS_TOL, _bias_before_bn, _fused_trainer

pytestmark = pytest.mark.gpu

ARCH, ZT, C, N, NL = "VAE64", 64, 3, 256, 4
HP = {"temperature": 0.1, "beta": 1 / 32, "loc": 0, "scale": 1, "alpha": 100.0, "lambda": 3.0}


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


def test_c3_mim_step_full_batch():
    from oracle import cpu_ref as R
    from cvhip import rng
    from cvhip.engine import ClearStep

    torch.set_num_threads(min(16, torch.get_num_threads()))
    sd = R.det_state(ARCH, ZT, C)
    x, label, ec, es, perm = R.det_inputs(N, C, 64, ZT, NL)
    tr = _fused_trainer(ARCH, ZT, C, sd, HP, mode="mim", kind="CLUBSample", lr=3e-5)
    eng = ClearStep.build(tr, "mim")
    assert eng is not None
    d = ZT // 2
    gen = np.random.default_rng(7)
    noises = [(ec, es)] + [(gen.standard_normal((N, d)), gen.standard_normal((N, d))) for _ in range(5)]
    rng.clear_injections()
    rng.inject_noise([torch.tensor(a, dtype=torch.float32) for pair in noises for a in pair])
    rng.inject_perm([torch.tensor(perm)])
    masks, grads = {}, {}

    def pin():  # gradients complete, Adam not yet run
        masks.update(device_masks(eng, eng.graphs[N]["ws"], N))
        for k, p in tr.model.named_parameters():
            grads[k] = p.grad.detach().double().cpu().clone()

    losses, learn = eng.step(torch.tensor(x, dtype=torch.float32, device="cuda"), torch.tensor(label, device="cuda"),
                             before_update=pin)
    losses, learn = losses.clone().cpu(), learn.cpu()
    assert masks and grads
    M = R.to_torch(R.det_mlp(d, ZT))
    args = (torch.tensor(x), torch.tensor(label), torch.tensor(ec), torch.tensor(es), torch.tensor(perm), ARCH, HP,
            "CLUBSample")
    o = R.mim_step(R.to_torch(sd), M, *args, masks=masks)
    for i, k in ((0, "rec"), (1, "kl_c"), (2, "kl_s"), (3, "c_loss")):
        assert abs(float(losses[i]) - float(o[k])) <= LOSS_TOL * max(abs(float(o[k])), 1e-3), (k, float(losses[i]),
                                                                                             float(o[k]))
    mi = float(o["mi"])
    assert abs(float(losses[5]) - mi) <= LOSS_TOL * max(abs(mi), 1.0), ("mi", float(losses[5]), mi)

    # mask-pinned gradients at the fp32 floor
    o32 = R.mim_step(R.to_torch(sd, torch.float32), R.to_torch(R.det_mlp(d, ZT), torch.float32),
                     torch.tensor(x, dtype=torch.float32), torch.tensor(label), torch.tensor(ec, dtype=torch.float32),
                     torch.tensor(es, dtype=torch.float32), torch.tensor(perm), ARCH, HP, "CLUBSample", masks=masks)
    rels, over = [], []
    for k, g in grads.items():
        g_ref = o["grads"][k].detach().numpy()
        if _bias_before_bn(k, ARCH):
            assert float(g.abs().max()) == 0.0, k
            continue
        r = _rel(g.numpy(), g_ref)
        floor = _rel(o32["grads"][k].detach().double().numpy(), g_ref)
        rels.append((r, k, floor))
        if r >= max(WORST_TOL, FLOOR_X * floor):
            over.append((k, r, floor))
    rels.sort()
    med = rels[len(rels) // 2][0]
    print(f"\nC3 n={N}: median {med:.2e}; worst (rel, tensor, fp32 floor): "
          + ", ".join(f"({r:.1e}, {k}, {f:.1e})" for r, k, f in rels[-3:]))
    assert med < MEDIAN_TOL, (med, rels[-3:])
    assert not over, over

    # the 5 estimator updates: the VAE after torch Adam on the oracle gradients (lr 3e-5), then per update a
    # train-mode forward with fresh noise, the learning loss and torch Adam on the estimator (lr 2e-3)
    P1 = R.to_torch(sd, requires_grad=False)
    names = list(o["grads"])
    vps = [P1[k].clone().requires_grad_(True) for k in names]
    for p_, k in zip(vps, names):
        p_.grad = torch.zeros_like(o["grads"][k]) if _bias_before_bn(k, ARCH) else o["grads"][k].detach().clone()
    torch.optim.Adam(vps, lr=3e-5).step()
    for p_, k in zip(vps, names):
        P1[k] = p_.detach()
    mparams = [M[k].detach().clone().requires_grad_(True) for k in M]
    Md = dict(zip(M.keys(), mparams))
    eopt = torch.optim.Adam(mparams, lr=2e-3)
    for j in range(5):
        a, b = noises[1 + j]
        with torch.no_grad():
            _, _, zz = R.vae_forward(P1, torch.tensor(x), torch.tensor(a), torch.tensor(b), ARCH, True)
        ll = R.learning_loss(Md, zz[:, :d], zz[:, d:])
        eopt.zero_grad()
        ll.backward()
        eopt.step()
        assert abs(float(learn[j]) - float(ll)) <= 1e-4 * max(abs(float(ll)), 1.0), (j, float(learn[j]), float(ll))
