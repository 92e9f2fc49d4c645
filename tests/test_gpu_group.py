"""GVAE / ML-VAE group evidence on the HIP path (reference code/src/models/vae.py:159-223,
code/src/trainer.py:291-353) against the fp64 oracle (oracle/cpu_ref.group_evidence / group_step, pinned to
the real reference by tests/golden/vae*_gvae*.npz / vae*_mlvae.npz).

Module path: accumulate_group_evidence (cv_group_forward + cv_group_evidence_backward) on ragged label sets
(gaps, negative and large label values, singleton groups, one group, n = 4096, and n = 8192 / 10000 above the
labels' LDS cache) — group rows 1e-5 relative
(fp32 segmented sums vs fp64), member dict bit-exact, input gradients 1e-4 relative.  Fused step
(HierarchicalVAETrainer, mode "group"): losses 1e-4 relative, VAE gradients by _check_grads, parameters
after Adam median < 1e-5 / worst < 5e-3, as tests/test_gpu_parity.py."""

import numpy as np
import pytest
import torch

from test_gpu_parity import LOSS_TOL, _bias_before_bn, _check_grads, _conditioning, _rel

pytestmark = pytest.mark.gpu


def _labels(n, kind, seed=0):
    g = np.random.default_rng(seed)
    if kind == "ragged":  # gaps, negative and large values, very unequal group sizes
        vals = np.array([-7, -1, 0, 3, 4, 11, 1000, 2 ** 40])
        p = np.array([0.4, 0.02, 0.2, 0.1, 0.08, 0.1, 0.05, 0.05])
        return vals[g.choice(len(vals), size=n, p=p)].astype(np.int64)
    if kind == "singletons":
        return g.permutation(n).astype(np.int64) * 3 - n
    if kind == "one":
        return np.full(n, 5, dtype=np.int64)
    return g.integers(0, 100, size=n).astype(np.int64)


@pytest.mark.parametrize("mode", ["GVAE", "MLVAE"])
@pytest.mark.parametrize("n,d,kind", [(64, 8, "ragged"), (257, 32, "ragged"), (40, 8, "singletons"),
                                      (16, 4, "one"), (4096, 8, "many"),
                                      # above the LDS label cache (group_forward_kernel<true>): no batch cap
                                      (8192, 8, "many"), (10000, 8, "ragged")])
def test_group_evidence_module(mode, n, d, kind):
    from oracle import cpu_ref as R
    from src.models.vae import accumulate_group_evidence

    g = np.random.default_rng(1)
    mu = g.standard_normal((n, d))
    lv = 0.5 * g.standard_normal((n, d))
    lab = _labels(n, kind)
    mu_t = torch.tensor(mu, dtype=torch.float32, device="cuda", requires_grad=True)
    lv_t = torch.tensor(lv, dtype=torch.float32, device="cuda", requires_grad=True)
    mu_g, lv_g, idx = accumulate_group_evidence(mu_t, lv_t, torch.tensor(lab, device="cuda"), mode)
    # oracle (fp64 inputs; the reference's fp32 group rows)
    mu_o = torch.tensor(mu, requires_grad=True)
    lv_o = torch.tensor(lv, requires_grad=True)
    mg_o, lg_o, idx_o = R.group_evidence(mu_o, lv_o, torch.tensor(lab), mode)
    assert list(idx) == list(idx_o)
    for k in idx:
        assert torch.equal(idx[k].cpu(), idx_o[k]), k
    assert _rel(mu_g, mg_o) < 1e-5 and _rel(lv_g, lg_o) < 1e-5, (_rel(mu_g, mg_o), _rel(lv_g, lg_o))
    A = g.standard_normal((len(idx), d))
    B = g.standard_normal((len(idx), d))
    ((mu_g * torch.tensor(A, dtype=torch.float32, device="cuda")).sum()
     + (lv_g * torch.tensor(B, dtype=torch.float32, device="cuda")).sum()).backward()
    ((mg_o * torch.tensor(A)).sum() + (lg_o * torch.tensor(B)).sum()).backward()
    assert _rel(mu_t.grad, mu_o.grad) < 1e-4, _rel(mu_t.grad, mu_o.grad)
    assert _rel(lv_t.grad, lv_o.grad) < 1e-4, _rel(lv_t.grad, lv_o.grad)


def test_groupwise_reparam_order():
    """groupwise_reparam_each: noise consumed in group order, z scattered back to batch order, and the
    reference's (indices, sizes) outputs."""
    from oracle import cpu_ref as R
    from cvhip import rng
    from src.models.vae import accumulate_group_evidence, groupwise_reparam_each

    n, d = 50, 8
    g = np.random.default_rng(2)
    mu, lv = g.standard_normal((n, d)), 0.3 * g.standard_normal((n, d))
    lab = _labels(n, "ragged", seed=3)
    eps = g.standard_normal((n, d))  # group-order rows
    mu_g, lv_g, idx = accumulate_group_evidence(torch.tensor(mu, dtype=torch.float32, device="cuda"),
                                                torch.tensor(lv, dtype=torch.float32, device="cuda"),
                                                torch.tensor(lab, device="cuda"), "MLVAE")
    rng.clear_injections()
    rng.inject_noise([torch.tensor(eps, dtype=torch.float32)])
    z, indices, sizes = groupwise_reparam_each(mu_g, lv_g, idx)
    mg_o, lg_o, idx_o = R.group_evidence(torch.tensor(mu), torch.tensor(lv), torch.tensor(lab), "MLVAE")
    z_o = R.group_reparam(mg_o, lg_o, idx_o, torch.tensor(eps))
    assert _rel(z, z_o) < 1e-5
    assert torch.equal(indices.cpu(), torch.cat(list(idx_o.values())))
    assert torch.equal(sizes.cpu(), torch.cat([torch.full((len(v),), len(v)) for v in idx_o.values()]))


def _group_trainer(arch, zt, C, sd, mode, lr):
    from src.models.vae import VAE, VAE64
    from src.trainer import HierarchicalVAETrainer

    vae = (VAE if arch == "VAE" else VAE64)(zt, C, group_mode=mode).cuda()
    vae.load_state_dict({k: torch.as_tensor(np.asarray(v)).float() if np.asarray(v).dtype != np.int64
                         else torch.as_tensor(np.asarray(v)) for k, v in sd.items()})
    opt = torch.optim.Adam(vae.parameters(), lr=lr)
    hp = {"beta": 0.125, "loc": 0, "scale": 1}
    return HierarchicalVAETrainer(vae, opt, hp, 1, torch.device("cuda")), hp


@pytest.mark.parametrize("mode", ["GVAE", "MLVAE"])
@pytest.mark.parametrize("arch,zt,C,n,nl", [("VAE", 16, 1, 64, 10), ("VAE", 16, 1, 256, 10),
                                            ("VAE", 16, 1, 48, 60), ("VAE64", 64, 3, 32, 4)])
def test_fused_group_step(mode, arch, zt, C, n, nl):
    from oracle import cpu_ref as R
    from cvhip import rng
    from cvhip.engine import ClearStep

    sd = R.det_state(arch, zt, C)
    x, label, ec, es, _ = R.det_inputs(n, C, R.IMAGE[arch], zt, nl)
    lr = 5e-4 if arch == "VAE" else 3e-5
    tr, hp = _group_trainer(arch, zt, C, sd, mode, lr)
    eng = ClearStep.build(tr, "group")
    assert eng is not None and eng.mode == "group", "group fused engine not built"
    ec_sorted = R.group_order_noise(label, torch.tensor(ec))
    rng.clear_injections()
    rng.inject_noise([ec_sorted.float(), torch.tensor(es, dtype=torch.float32)])
    losses = eng.step(torch.tensor(x, dtype=torch.float32, device="cuda"), torch.tensor(label, device="cuda"))
    losses = losses.clone().cpu()

    def step(xx):
        return R.group_step(R.to_torch(sd), torch.tensor(xx), torch.tensor(label), ec_sorted, torch.tensor(es), arch,
                            hp, mode)

    o = step(x)
    for i, k in ((0, "rec_adj"), (1, "kl_c"), (2, "kl_s_adj")):
        ref = float(o[k].detach())
        assert abs(float(losses[i]) - ref) <= LOSS_TOL * max(abs(ref), 1e-3), (k, float(losses[i]), ref)
    _check_grads({k: p.grad for k, p in tr.model.named_parameters()}, o["grads"], arch, _conditioning(o, step, x))
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
    # a graph-replayed step on Philox noise: finite losses, the annealer and Adam counters advance
    losses2 = eng.step(torch.tensor(x, dtype=torch.float32, device="cuda"), torch.tensor(label, device="cuda"))
    losses3 = eng.step(torch.tensor(x, dtype=torch.float32, device="cuda"), torch.tensor(label, device="cuda"))
    assert torch.isfinite(losses3[:3]).all()
    eng.sync_host_state()
    assert int(float(tr.optimizer.state[next(tr.model.parameters())]["step"])) == 3


def test_group_fit_through_factory():
    """get_hierarchical_vae_trainer(...).fit trains on the fused path; evaluate() with evidence runs the
    module path."""
    from oracle import cpu_ref as R
    from src.utils.trainer_utils import get_hierarchical_vae_trainer

    torch.manual_seed(0)
    tr = get_hierarchical_vae_trainer(beta=1 / 8, vae_lr=5e-4, z_dim=16, group_mode="MLVAE", device="cuda",
                                      verbose_period=100)
    x, label, _, _, _ = R.det_inputs(512, 1, 28, 16, 10, seed=9)
    ds = torch.utils.data.TensorDataset(torch.tensor(x, dtype=torch.float32), torch.tensor(label))
    dl = torch.utils.data.DataLoader(ds, batch_size=128, shuffle=False)
    tr.fit(1, dl)
    assert tr._engine is not None and tr._engine.mode == "group", "fused group engine not used"
    first = tr._engine.last_workspace(128).losses.clone()
    tr.fit(6, dl)
    last = tr._engine.last_workspace(128).losses.clone()
    assert float(last[0]) < float(first[0])
    mig, mse = tr.evaluate(dl, False, 0, with_evidence_acc=True)
    assert np.isfinite(mse)
