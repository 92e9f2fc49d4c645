"""Pin the oracle (oracle/cpu_ref.py) to the real reference: every golden fixture (one real trainer step
of scotsun/clear-vae in fp64, tests/golden/gen_golden.py) is recomputed by the oracle in fp64 on the
same inputs and must agree to 1e-9 relative (fp64 vs fp64; the only differences are summation
orders inside ATen).  CPU only."""

import numpy as np
import pytest
import torch

import golden_cases as G

TOL = 1e-9


@pytest.fixture(scope="module", params=G.names())
def case(request):
    fx = G.load(request.param)
    torch.set_num_threads(4)
    return request.param, fx, G.oracle_step(fx)


def test_fixture_set_complete():
    have = set(G.names())
    for need in ("vae_n64_cosine_ps1", "vae_n64_cosine_ps0", "vae_n64_l2_ps1", "vae_n64_jeffrey_ps1",
                 "vae_n512_cosine_ps1", "vae_n64_mim_club", "vae_n64_mim_l1out", "vae64_n16_cosine_ps1",
                 "vae64_n16_mim_club", "vae_n64_tc", "vae64_n16_tc", "vae_n64_gvae", "vae_n64_mlvae",
                 "vae_n32_gvae_l40", "vae64_n16_mlvae"):
        assert need in have, need


def test_losses_and_latents(case):
    name, fx, o = case
    mode = fx["meta"]["mode"]
    for k in ("rec", "kl_c", "kl_s") + (("c_loss",) if mode != "group" else ()):
        assert abs(o[k] - float(fx[k])) <= TOL * max(abs(float(fx[k])), 1e-3), (name, k, o[k], float(fx[k]))
    if mode == "clear":
        assert abs(o["s_loss"] - float(fx["s_loss"])) <= TOL * max(abs(float(fx["s_loss"])), 1e-3)
    elif mode == "group":  # number of groups, and z = grouped reparam | per-sample reparam
        assert o["m"] == int(fx["m"])
        assert G.rel(o["z"], fx["z"]) < TOL
    else:
        # the MI term is signed and can be near zero: relative + absolute floor
        assert abs(o["mi"] - float(fx["mi"])) <= TOL * max(abs(float(fx["mi"])), 1.0)
        assert G.rel(o["z"], fx["z"]) < TOL
    for k in ("mu_c", "logvar_c", "mu_s", "logvar_s"):
        assert G.rel(o[k], fx[k]) < TOL, (name, k)
    if "xhat" in fx:
        assert G.rel(o["xhat"], fx["xhat"]) < 1e-7  # stored as fp32


def test_gradients(case):
    name, fx, o = case
    # biases feeding a train-mode BatchNorm have an analytically zero gradient (both sides are
    # rounding noise there): an absolute floor at 1e-10 of the largest gradient norm covers them
    gmax = max(float(fx["gnorm__" + k]) for k in o["grads"])
    for k, g in o["grads"].items():
        gn = float(fx["gnorm__" + k])
        assert abs(np.linalg.norm(g) - gn) <= 1e-8 * gn + 1e-10 * gmax, (name, k)
        ours, ref = G.pick(fx, "grad__", k, g)
        err = np.linalg.norm(np.asarray(ours) - ref)
        assert err <= 1e-8 * np.linalg.norm(ref) + 1e-10 * gmax, (name, k, err, np.linalg.norm(ref))


def test_adam_update_and_buffers(case):
    name, fx, o = case
    lr = fx["meta"]["hp"]["lr"]
    for k, p in o["after"].items():
        ours, ref = G.pick(fx, "after__", k, p)
        # Adam's first step is lr*g/(|g|+eps): for the rounding-noise gradients of biases feeding a
        # train-mode BN the step itself is noise, so those are held to 1e-4 of lr in absolute terms
        assert G.rel(ours, ref) < 1e-9 or np.abs(ours - ref).max() <= 1e-4 * lr, (name, k)
    # CLEAR-MIM's 5 extra forwards run on the post-Adam weights, so the running means inherit the
    # noise-level bias steps above (the conv bias shifts the BN input mean one-for-one)
    btol = 1e-9 if fx["meta"]["mode"] in ("clear", "group") else 1e-7  # (CLEAR-TC: one extra forward, as MIM)
    for k, b in o["buffers"].items():
        assert G.rel(b, fx["buf__" + k]) < btol, (name, k)
    if fx["meta"]["mode"] == "mim":
        assert np.allclose(o["mi_learning"], fx["mi_learning"], rtol=1e-9, atol=1e-9), (o["mi_learning"],
                                                                                       fx["mi_learning"])
        for k, v in o["est_after"].items():
            assert G.rel(v, fx["est_after__" + k]) < 1e-9, (name, k)


def test_clear_tc_factor_step(case):
    """CLEAR-TC's factor-discriminator step (trainer.py:680-699): z of the second forward, the BCE value,
    the discriminator gradients and its parameters after torch Adam."""
    name, fx, o = case
    if fx["meta"]["mode"] != "tc":
        pytest.skip("CLEAR-TC cases only")
    assert G.rel(o["z2"], fx["z2"]) < 1e-7  # post-Adam weights: the bias-noise steps above
    assert abs(o["factor_loss"] - float(fx["factor_loss"])) <= 1e-7 * abs(float(fx["factor_loss"]))
    for k, g in o["disc_grad"].items():
        assert G.rel(g, fx["disc_grad__" + k]) < 1e-6, (name, k)
    for k, v in o["disc_after"].items():
        assert G.rel(v, fx["disc_after__" + k]) < 1e-9, (name, k)


def test_bf16_conv_restatement():
    """oracle/cpu_ref.py _Bf16Conv (the bf16 GEMM-core arithmetic the bf16 tests pin against): with operands
    and incoming gradient already bf16-representable it is the plain fp64 conv / convT with its exact autograd;
    otherwise it differs by bf16 rounding of exactly those three tensors."""
    import torch.nn.functional as F

    from oracle import cpu_ref as R

    g = torch.Generator().manual_seed(0)
    for transposed in (False, True):
        h = torch.randn(2, 8, 6, 6, generator=g, dtype=torch.float64)
        w = torch.randn(8, 4, 3, 3, generator=g, dtype=torch.float64) if transposed else \
            torch.randn(4, 8, 3, 3, generator=g, dtype=torch.float64)
        b = torch.randn(4, generator=g, dtype=torch.float64)
        op = 1 if transposed else 0
        for exact in (True, False):
            hh, ww = (R._r16(h), R._r16(w)) if exact else (h, w)
            a1, w1, b1 = (t.clone().requires_grad_(True) for t in (hh, ww, b))
            y = R._Bf16Conv.apply(a1, w1, b1, 2, 1, op, transposed)
            gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
            gy = R._r16(gy) if exact else gy
            y.backward(gy)
            a2, w2, b2 = (t.clone().requires_grad_(True) for t in (R._r16(hh), R._r16(ww), b))
            f = (lambda u, v, c: F.conv_transpose2d(u, v, c, stride=2, padding=1, output_padding=1)) if transposed \
                else (lambda u, v, c: F.conv2d(u, v, c, stride=2, padding=1))
            y2 = f(a2, w2, b2)
            y2.backward(R._r16(gy))
            assert torch.allclose(y, y2, rtol=1e-12, atol=1e-12)
            assert torch.allclose(a1.grad, a2.grad, rtol=1e-12, atol=1e-12)
            assert torch.allclose(w1.grad, w2.grad, rtol=1e-12, atol=1e-12)
            assert torch.allclose(b1.grad, gy.sum(dim=(0, 2, 3)))
            if not exact:  # the rounding is really in effect
                y3 = f(h, w, b)
                assert float((y3 - y).abs().max()) > 1e-4


@pytest.mark.parametrize("sim_fn", ["cosine", "l2", "jeffrey", "mahalanobis", "modified_l2"])
@pytest.mark.parametrize("ps", [False, True])
def test_blockwise_contrastive_matches_reference_form(sim_fn, ps):
    """oracle.cpu_ref.contrastive_loss_blockwise (the large-batch restatement used at N = 8192) against the
    literal restatement of losses.py:98-126 at N = 96, value and gradient (fp64, 1e-12)."""
    from oracle import cpu_ref as R

    g = torch.Generator().manual_seed(3)
    n, d = 96, 8
    mu = torch.randn(n, d, generator=g, dtype=torch.float64)
    lv = 0.3 * torch.randn(n, d, generator=g, dtype=torch.float64)
    label = torch.randint(0, 4, (n,), generator=g)
    label[5] = 99  # a singleton: an all -inf positive row (dropped by the finite-row mean when ps=False)
    m1, l1 = mu.clone().requires_grad_(True), lv.clone().requires_grad_(True)
    ref = R.contrastive_loss(m1, l1, label, sim_fn, 0.3, ps)
    ref.backward()
    m2, l2 = mu.clone().requires_grad_(True), lv.clone().requires_grad_(True)
    got = R.contrastive_loss_blockwise(m2, l2, label, sim_fn, 0.3, ps, block=17)
    assert abs(float(got) - float(ref)) <= 1e-12 * max(1.0, abs(float(ref)))
    assert torch.allclose(m2.grad, m1.grad, rtol=1e-10, atol=1e-12)
    if l1.grad is not None:
        assert torch.allclose(l2.grad, l1.grad, rtol=1e-10, atol=1e-12)


def test_l1out_closed_form_matches_broadcast():
    """oracle.cpu_ref.l1out_closed against the literal [N,N,N] restatement (mi_estimator.py:170-191) at N = 48."""
    from oracle import cpu_ref as R

    g = torch.Generator().manual_seed(4)
    M = R.to_torch(R.det_mlp(8, 16))
    x = torch.randn(48, 8, generator=g, dtype=torch.float64, requires_grad=True)
    y = torch.randn(48, 8, generator=g, dtype=torch.float64, requires_grad=True)
    a = R.l1out(M, x, y)
    b = R.l1out_closed(M, x, y)
    assert abs(float(a) - float(b)) <= 1e-11 * max(1.0, abs(float(a)))
    ga = torch.autograd.grad(a, (x, y))
    gb = torch.autograd.grad(b, (x, y))
    for u, v in zip(ga, gb):
        assert torch.allclose(u, v, rtol=1e-9, atol=1e-12)
