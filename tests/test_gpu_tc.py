"""CLEAR-TC on the fused engine (reference code/src/trainer.py:590-778,
code/src/utils/trainer_utils.py:119-157) against the fp64 oracle (oracle/cpu_ref.tc_step / tc_factor_loss,
pinned to the real reference by tests/golden/vae*_tc.npz).

One step = the VAE step with lambda * relu(log(D/(1-D))).mean() of the factor discriminator D, torch Adam
semantics on the VAE, a second train-mode forward with fresh noise on the updated VAE, and D's BCE step on
joint vs factor-shuffled z with its own Adam.  Tolerances as tests/test_gpu_parity.py: losses and the
density-ratio term 1e-4 relative (absolute floor 1 for the signed term), VAE gradients by _check_grads,
parameters after Adam median < 1e-5 / worst < 5e-3; the discriminator step runs downstream of the VAE's
Adam step (whose noise-gradient biases move by ~lr either way), so its loss / gradients / parameters are
held to 1e-3."""

import numpy as np
import pytest
import torch

from test_gpu_parity import LOSS_TOL, _bias_before_bn, _check_grads, _model, _rel

pytestmark = pytest.mark.gpu


def _tc_trainer(arch, zt, C, sd, hp, lr, flr):
    from oracle import cpu_ref as R
    from src.trainer import ClearTCVAETrainer

    vae = _model(arch, zt, C, sd)
    opt = torch.optim.Adam(vae.parameters(), lr=lr)
    disc = torch.nn.Sequential(torch.nn.Linear(zt, zt), torch.nn.ReLU(), torch.nn.Linear(zt, 1),
                               torch.nn.Sigmoid()).cuda()
    disc.load_state_dict({k: torch.tensor(v, dtype=torch.float32) for k, v in R.det_disc(zt).items()})
    fopt = torch.optim.Adam(disc.parameters(), lr=flr)
    return ClearTCVAETrainer(vae, disc, {"vae_optim": opt, "factor_optim": fopt}, "cosine", hp, 1,
                             torch.device("cuda"))


@pytest.mark.parametrize("arch,zt,C,n", [("VAE", 16, 1, 64), ("VAE", 16, 1, 256), ("VAE64", 64, 3, 32)])
def test_fused_tc_step(arch, zt, C, n):
    from oracle import cpu_ref as R
    from cvhip import rng
    from cvhip.engine import ClearStep

    sd = R.det_state(arch, zt, C)
    x, label, ec, es, _ = R.det_inputs(n, C, R.IMAGE[arch], zt, 10)
    gen = np.random.default_rng(6)
    a, b = gen.standard_normal((n, zt // 2)), gen.standard_normal((n, zt // 2))
    lr, flr = (5e-4 if arch == "VAE" else 3e-5), 1e-3
    hp = {"temperature": 0.1, "alpha": 100.0, "beta": 0.125, "loc": 0, "scale": 1, "lambda": 3.0}
    tr = _tc_trainer(arch, zt, C, sd, hp, lr, flr)
    eng = ClearStep.build(tr, "tc")
    assert eng is not None, "CLEAR-TC fused engine not built"
    rng.clear_injections()
    rng.inject_noise([torch.tensor(t, dtype=torch.float32) for t in (ec, es, a, b)])
    losses, fl = eng.step(torch.tensor(x, dtype=torch.float32, device="cuda"), torch.tensor(label, device="cuda"))
    losses, fl = losses.clone().cpu(), float(fl)
    # oracle: VAE half
    D = R.to_torch(R.det_disc(zt))
    o = R.tc_step(R.to_torch(sd), D, torch.tensor(x), torch.tensor(label), torch.tensor(ec), torch.tensor(es), arch, hp)
    for i, k in ((0, "rec"), (1, "kl_c"), (2, "kl_s"), (3, "c_loss")):
        ref = float(o[k].detach())
        assert abs(float(losses[i]) - ref) <= LOSS_TOL * max(abs(ref), 1e-3), (k, float(losses[i]), ref)
    mi = float(o["mi"].detach())
    assert abs(float(losses[5]) - mi) <= LOSS_TOL * max(abs(mi), 1.0), (float(losses[5]), mi)
    _check_grads({k: p.grad for k, p in tr.model.named_parameters()}, o["grads"], arch)
    # VAE parameters after Adam
    P1 = R.to_torch(sd, requires_grad=False)
    names = list(o["grads"])
    vps = [P1[k].clone().requires_grad_(True) for k in names]
    for p_, k in zip(vps, names):
        p_.grad = torch.zeros_like(o["grads"][k]) if _bias_before_bn(k, arch) else o["grads"][k].clone()
    torch.optim.Adam(vps, lr=lr).step()
    cur = dict(tr.model.named_parameters())
    prel = sorted((_rel(cur[k], p_), k) for p_, k in zip(vps, names))
    assert prel[len(prel) // 2][0] < 1e-5, prel[-3:]
    assert prel[-1][0] < 5e-3, prel[-3:]
    # oracle: discriminator step on the second forward's z
    for p_, k in zip(vps, names):
        P1[k] = p_.detach()
    with torch.no_grad():
        _, _, z2 = R.vae_forward(P1, torch.tensor(x), torch.tensor(a), torch.tensor(b), arch, True)
    Dp = [v.detach().clone().requires_grad_(True) for v in D.values()]
    Dd = dict(zip(D.keys(), Dp))
    flo = R.tc_factor_loss(Dd, z2)
    flo.backward()
    assert abs(fl - float(flo)) <= 1e-3 * abs(float(flo)), (fl, float(flo))
    torch.optim.Adam(Dp, lr=flr).step()
    for k, p in tr.factor_cls.named_parameters():
        assert _rel(p, Dd[k]) < 1e-3, k
    eng.sync_host_state()
    assert int(float(tr.factor_optimizer.state[next(tr.factor_cls.parameters())]["step"])) == 1


def test_tc_fit_through_factory():
    """get_cleartcvae_trainer(...).fit: the fused path trains and returns one factor loss per step."""
    from oracle import cpu_ref as R
    from src.utils.trainer_utils import get_cleartcvae_trainer

    torch.manual_seed(0)
    tr = get_cleartcvae_trainer(beta=1 / 8, la=3.0, vae_lr=5e-4, factor_cls_lr=1e-3, z_dim=16, alpha=100,
                                temperature=0.1, device="cuda", verbose_period=100)
    x, label, _, _, _ = R.det_inputs(512, 1, 28, 16, 10, seed=9)
    ds = torch.utils.data.TensorDataset(torch.tensor(x, dtype=torch.float32), torch.tensor(label))
    dl = torch.utils.data.DataLoader(ds, batch_size=128, shuffle=False)
    fl = tr.fit(1, dl)
    assert tr._engine is not None and tr._engine.mode == "tc", "fused CLEAR-TC engine not used"
    first = tr._engine.last_workspace(128).losses.clone()
    fl += tr.fit(6, dl)
    last = tr._engine.last_workspace(128).losses.clone()
    assert len(fl) == 7 * 4 and all(np.isfinite(fl))
    assert float(last[0]) < float(first[0])
