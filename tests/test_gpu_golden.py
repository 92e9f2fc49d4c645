"""The HIP path against the committed golden fixtures (one real reference trainer step each, fp64,
tests/golden/gen_golden.py): the module path for the model outputs (latents, z, x_hat, losses, MI)
and the fused trainer step for the trainer-level results (losses, gradients, parameters after Adam,
BN running statistics, CLEAR-MIM estimator learning losses).

Tolerances as in test_gpu_parity.py: outputs 1e-4 relative (the north_star bar; the signed MI term
with an absolute floor); gradients median per-tensor < 5e-4 / worst < 2e-2 on the stored samples
(knife-edge ReLU flips, see that module's docstring); parameters after Adam: median < 1e-5, worst
< 5e-3 (Adam's first step is ~lr*sign(g)).  Biases that feed a train-mode BatchNorm: exact zero
gradient on the HIP path vs rounding noise in the reference, so their Adam step is compared to lr."""

import numpy as np
import pytest
import torch

import golden_cases as G

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _model(fx):
    from oracle import cpu_ref as R
    from src.models.vae import VAE, VAE64

    m = fx["meta"]
    gm = m["estimator"] if m["mode"] == "group" else None
    vae = (VAE if m["arch"] == "VAE" else VAE64)(m["z"], m["C"], group_mode=gm).cuda()
    sd = R.det_state(m["arch"], m["z"], m["C"])
    vae.load_state_dict({k: torch.as_tensor(np.asarray(v)).float() if np.asarray(v).dtype != np.int64
                         else torch.as_tensor(np.asarray(v)) for k, v in sd.items()})
    return vae


def _estimator(fx):
    from oracle import cpu_ref as R
    from src.models.mi_estimator import CLUBSample, L1OutUB

    m = fx["meta"]
    d = m["z"] // 2
    est = (CLUBSample if m["estimator"] == "CLUBSample" else L1OutUB)(d, d, m["z"]).cuda()
    est.load_state_dict({k: torch.tensor(v, dtype=torch.float32) for k, v in R.det_mlp(d, m["z"]).items()})
    return est


def _disc(fx):
    from oracle import cpu_ref as R

    z = fx["meta"]["z"]
    disc = torch.nn.Sequential(torch.nn.Linear(z, z), torch.nn.ReLU(), torch.nn.Linear(z, 1), torch.nn.Sigmoid()).cuda()
    disc.load_state_dict({k: torch.tensor(v, dtype=torch.float32) for k, v in R.det_disc(z).items()})
    return disc


def _close(a, ref, floor=1e-3):
    return abs(float(a) - float(ref)) <= TOL * max(abs(float(ref)), floor)


def _bias_before_bn(name, arch):
    from oracle import cpu_ref as R

    parts = name.split(".")
    return (parts[-1] == "bias" and parts[0] in ("encoder", "decoder")
            and R._layer_kind(arch, parts[0], int(parts[1])) in ("conv", "linear"))


@pytest.mark.parametrize("name", G.names())
def test_module_outputs_vs_golden(name):
    from cvhip import rng
    from src.losses import contrastive_loss, vae_loss

    fx = G.load(name)
    m = fx["meta"]
    x, label, ec, es, perm = G.inputs(fx)
    vae = _model(fx)
    vae.train()
    X = torch.tensor(x, dtype=torch.float32, device="cuda")
    L = torch.tensor(label, device="cuda")
    rng.clear_injections()
    if m["mode"] == "group":  # vae(X, label): group evidence, content noise consumed in group order
        from oracle import cpu_ref as R

        rng.inject_noise([R.group_order_noise(label, torch.tensor(ec)).float(), torch.tensor(es, dtype=torch.float32)])
        with torch.no_grad():
            xhat, lp, z = vae(X, label=L, explicit=True)
            rec, kl_c, kl_s = vae_loss(xhat, X, **lp)
        for k in ("mu_c", "logvar_c", "mu_s", "logvar_s"):  # (mu_c / logvar_c: the m group rows)
            assert G.rel(lp[k].cpu().numpy(), fx[k]) < TOL, k
        assert G.rel(z.cpu().numpy(), fx["z"]) < TOL
        if "xhat" in fx:
            assert G.rel(xhat.cpu().numpy(), fx["xhat"]) < TOL
        for k, v in (("rec", rec), ("kl_c", kl_c), ("kl_s", kl_s)):
            assert _close(v, fx[k]), (k, float(v), float(fx[k]))
        return
    rng.inject_noise([torch.tensor(ec, dtype=torch.float32), torch.tensor(es, dtype=torch.float32)])
    with torch.no_grad():
        xhat, lp, z = vae(X, explicit=True)
        rec, kl_c, kl_s = vae_loss(xhat, X, **lp)
        c = contrastive_loss(lp["mu_c"], lp["logvar_c"], L, m["sim_fn"], m["hp"]["temperature"])
    for k in ("mu_c", "logvar_c", "mu_s", "logvar_s"):
        assert G.rel(lp[k].cpu().numpy(), fx[k]) < TOL, k
    if "xhat" in fx:
        assert G.rel(xhat.cpu().numpy(), fx["xhat"]) < TOL
    for k, v in (("rec", rec), ("kl_c", kl_c), ("kl_s", kl_s), ("c_loss", c)):
        assert _close(v, fx[k]), (k, float(v), float(fx[k]))
    if m["mode"] == "clear":
        with torch.no_grad():
            s = contrastive_loss(lp["mu_s"], lp["logvar_s"], L, m["sim_fn"], m["hp"]["temperature"], ps=m["ps"])
        assert _close(s, fx["s_loss_raw"]), (float(s), float(fx["s_loss_raw"]))
    elif m["mode"] == "tc":
        assert G.rel(z.cpu().numpy(), fx["z"]) < TOL
        with torch.no_grad():
            dsc = _disc(fx)(z)
            mi = torch.relu(torch.log(dsc / (1 - dsc))).mean()
        assert abs(float(mi) - float(fx["mi"])) <= TOL * max(abs(float(fx["mi"])), 1.0), (float(mi), float(fx["mi"]))
    else:
        assert G.rel(z.cpu().numpy(), fx["z"]) < TOL
        est = _estimator(fx)
        rng.inject_perm([torch.tensor(perm)])
        d = m["z"] // 2
        with torch.no_grad():
            mi = est(z[:, :d], z[:, d:])
        assert abs(float(mi) - float(fx["mi"])) <= TOL * max(abs(float(fx["mi"])), 1.0), (float(mi), float(fx["mi"]))


def build_fused(fx):
    """The fixture's trainer and fused engine, with the case's noise (and CLUB-S permutation) queued for the
    next step.  Returns (trainer, engine, disc or None)."""
    from cvhip import rng
    from cvhip.engine import ClearStep
    from src.trainer import ClearMIMVAETrainer, ClearTCVAETrainer, CLEARVAETrainer, HierarchicalVAETrainer

    m = fx["meta"]
    x, label, ec, es, perm = G.inputs(fx)
    hp = G.hyper(fx)
    vae = _model(fx)
    disc = None
    opt = torch.optim.Adam(vae.parameters(), lr=hp["lr"])
    rng.clear_injections()
    noise = [torch.tensor(ec, dtype=torch.float32), torch.tensor(es, dtype=torch.float32)]
    if m["mode"] == "group":
        from oracle import cpu_ref as R

        tr = HierarchicalVAETrainer(vae, opt, {k: hp[k] for k in ("beta", "loc", "scale")}, 1, torch.device("cuda"))
        eng = ClearStep.build(tr, "group")
        noise[0] = R.group_order_noise(label, torch.tensor(ec)).float()
    elif m["mode"] == "clear":
        tr = CLEARVAETrainer(vae, opt, m["sim_fn"], hp, 1, torch.device("cuda"))
        eng = ClearStep.build(tr, "clear")
    elif m["mode"] == "tc":
        disc = _disc(fx)
        fopt = torch.optim.Adam(disc.parameters(), lr=hp["factor_lr"])
        tr = ClearTCVAETrainer(vae, disc, {"vae_optim": opt, "factor_optim": fopt}, m["sim_fn"], hp, 1,
                               torch.device("cuda"))
        eng = ClearStep.build(tr, "tc")
        for a, b in fx["extra_noise"]:
            noise += [torch.tensor(a, dtype=torch.float32), torch.tensor(b, dtype=torch.float32)]
    else:
        est = _estimator(fx)
        eopt = torch.optim.Adam(est.parameters(), lr=hp["est_lr"])
        tr = ClearMIMVAETrainer(vae, est, {"vae_optim": opt, "mi_estimator_optim": eopt}, m["sim_fn"], hp, 1,
                                torch.device("cuda"))
        eng = ClearStep.build(tr, "mim")
        for a, b in fx["extra_noise"]:
            noise += [torch.tensor(a, dtype=torch.float32), torch.tensor(b, dtype=torch.float32)]
        rng.inject_perm([torch.tensor(perm)])
    assert eng is not None
    rng.inject_noise(noise)
    return tr, eng, disc


@pytest.mark.parametrize("name", G.names())
def test_fused_step_vs_golden(name):
    fx = G.load(name)
    m = fx["meta"]
    arch = m["arch"]
    x, label, ec, es, perm = G.inputs(fx)
    hp = G.hyper(fx)
    tr, eng, disc = build_fused(fx)
    X = torch.tensor(x, dtype=torch.float32, device="cuda")
    out = eng.step(X, torch.tensor(label, device="cuda"))
    losses, learn = (out, None) if m["mode"] in ("clear", "group") else out
    losses = losses.clone().cpu()
    torch.cuda.synchronize()
    if m["mode"] == "group":  # the trainer's values: rec and kl_s after _group_adjust (x B/m)
        adj = m["n"] / int(fx["m"])
        for i, k, f in ((0, "rec", adj), (1, "kl_c", 1.0), (2, "kl_s", adj)):
            assert _close(losses[i], f * float(fx[k])), (k, float(losses[i]), f * float(fx[k]))
    else:
        for i, k in ((0, "rec"), (1, "kl_c"), (2, "kl_s"), (3, "c_loss")):
            assert _close(losses[i], fx[k]), (k, float(losses[i]), float(fx[k]))
    if m["mode"] == "group":
        pass
    elif m["mode"] == "clear":
        assert _close(losses[4], fx["s_loss_raw"]), (float(losses[4]), float(fx["s_loss_raw"]))
    elif m["mode"] == "tc":
        assert abs(float(losses[5]) - float(fx["mi"])) <= TOL * max(abs(float(fx["mi"])), 1.0)
        # the discriminator's step runs on z of a second forward through the post-Adam VAE, whose
        # knife-edge / noise-gradient Adam steps (see above) move z at ~1e-5: 1e-3 on its results
        assert abs(float(learn[0]) - float(fx["factor_loss"])) <= 1e-3 * abs(float(fx["factor_loss"]))
        dprels = []
        for k, p in disc.named_parameters():
            dprels.append(G.rel(p.detach().double().cpu().numpy(), fx["disc_after__" + k]))
        assert max(dprels) < 1e-3, dprels
    else:
        assert abs(float(losses[5]) - float(fx["mi"])) <= TOL * max(abs(float(fx["mi"])), 1.0)
        ll = learn.cpu().numpy()
        assert np.allclose(ll, fx["mi_learning"], rtol=1e-3, atol=1e-3), (ll, fx["mi_learning"])
    # gradients (the arena the Adam kernel consumed) on the stored samples
    rels = []
    lr = hp["lr"]
    for k, p in tr.model.named_parameters():
        g = p.grad.detach().double().cpu().numpy()
        ours, ref = G.pick(fx, "grad__", k, g)
        if _bias_before_bn(k, arch):
            assert np.abs(ours).max() == 0.0, k
            continue
        rels.append((G.rel(ours, ref), k))
    rels.sort()
    floor = 0.0
    if m["mode"] == "group":  # decoder-dominated gradients: bar at the reference's own knife-edge sensitivity
        from oracle import cpu_ref as R
        from test_gpu_parity import _conditioning

        Ecs = R.group_order_noise(label, torch.tensor(ec))

        def step(xx):
            return R.group_step(R.to_torch(R.det_state(arch, m["z"], m["C"])), torch.tensor(xx), torch.tensor(label),
                                Ecs, torch.tensor(es), arch, hp, m["estimator"])

        floor = _conditioning(step(x), step, x)[0]
    assert rels[len(rels) // 2][0] < max(5e-4, 2 * floor), (rels[-3:], floor)
    assert rels[-1][0] < 2e-2, rels[-3:]
    # parameters after the trainer's Adam step
    prels = []
    for k, p in tr.model.named_parameters():
        ours, ref = G.pick(fx, "after__", k, p.detach().double().cpu().numpy())
        if _bias_before_bn(k, arch):
            assert np.abs(ours - ref).max() <= 2.5 * lr, k
            continue
        prels.append((G.rel(ours, ref), k))
    prels.sort()
    assert prels[len(prels) // 2][0] < 1e-5, prels[-3:]
    assert prels[-1][0] < 5e-3, prels[-3:]
    # BatchNorm running statistics after the step's train-mode forwards (1, or 6 in CLEAR-MIM)
    btol = 1e-4 if m["mode"] in ("clear", "group") else 1e-3  # (MIM / TC: forwards after the Adam step)
    for k, v in tr.model.state_dict().items():
        if k.endswith(("running_mean", "running_var")):
            assert G.rel(v.double().cpu().numpy(), fx["buf__" + k]) < btol, k
        elif k.endswith("num_batches_tracked"):
            assert int(v) == int(fx["buf__" + k]), k
