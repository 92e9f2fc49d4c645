"""The fused engine's data-parallel step (cvhip/engine.py `_segments` / `make_learn_dp`), run as two
processes on the one GPU over gloo (tests/dp_gpu_worker.py), against the DDP semantics of SURVEY §8(e):

  * both ranks start from rank 0's parameters (rank 1 is built from different weights);
  * each rank runs the step on its contiguous half of the global batch (local-batch BN / contrastive /
    MI terms): its losses match the oracle on that shard;
  * the gradient both ranks apply is the mean of the per-shard oracle gradients;
  * the parameters after Adam are identical (bitwise) across ranks, equal to torch Adam applied to that
    mean gradient, and stay identical through graph-captured replays;
  * CLEAR-MIM: the estimator's 5 updates use the mean of the per-shard learning-loss gradients, and the
    estimator parameters are identical across ranks;
  * CLEAR-TC: the discriminator's BCE gradients are averaged the same way, its parameters identical across
    ranks; GVAE / ML-VAE: each rank's group evidence is over its own shard (the groups of its local batch).

Losses are held at 1e-4 relative (tests/test_gpu_parity.py).  Gradients are held mask-pinned
(tests/test_gpu_maskpinned.py): each rank reads the ReLU activity its shard's forward chose (tests/maskpin.py,
before Adam moves the BN affine), and the averaged gradient is compared, tensor by tensor, with the mean of the
per-shard fp64 oracle gradients evaluated with those masks — every tensor within max(1e-5, 8 x its fp32 floor),
the floor being the same pinned mean evaluated in fp32 (a cancelling batch sum carries that error in any fp32
evaluation), the median tensor within 5e-6.  The bf16 step is pinned the same way against the oracle that also
rounds the GEMM-core operands to bf16 where the kernels do (oracle/cpu_ref.py `bf16=`), held at the fp32 floor of
that function (tests/test_gpu_bf16.py `_check_bf16_pinned`: every tensor within max(1e-3, 2 x its floor))."""

import multiprocessing as mp
import socket

import numpy as np
import pytest
import torch

import dp_gpu_worker
from maskpin import masks_from_numpy
from test_gpu_parity import LOSS_TOL, _bias_before_bn

# mask-pinned gradient bars (fp32: tests/test_gpu_maskpinned.py; bf16: tests/test_gpu_bf16.py)
PIN = {"fp32": (5e-6, 1e-5)}  # (median tensor, every tensor at least); bf16: tests/test_gpu_bf16.py's floor bars
FLOOR_X = 8.0

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(mode, n_global, kind="CLUBSample", world=2, timeout=100, arch="VAE", precision="fp32"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=dp_gpu_worker.run, args=(r, world, port, q, mode, n_global, kind, arch, precision))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, out, err = q.get(timeout=timeout)
            assert err is None, err
            res[r] = out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return res


def _adam_ref(sd, grads, lr=5e-4, arch="VAE"):
    from oracle import cpu_ref as R

    P0 = R.to_torch(sd, requires_grad=False)
    names = list(grads)
    ps = [P0[k].clone().requires_grad_(True) for k in names]
    for p_, k in zip(ps, names):
        p_.grad = torch.zeros_like(grads[k]) if _bias_before_bn(k, arch) else grads[k].clone()
    torch.optim.Adam(ps, lr=lr).step()
    return {k: p_.detach() for k, p_ in zip(names, ps)}


def _rel(a, b):
    a, b = torch.as_tensor(a).double().reshape(-1), torch.as_tensor(b).double().reshape(-1)
    return float((a - b).norm() / (b.norm() + 1e-30))


def _check_pinned(res, shard_step, arch, precision="fp32"):
    """The averaged gradient (res[0]["grad"], = res[1]'s) against the mean of the per-shard mask-pinned oracle
    gradients: shard_step(r, dtype, masks) -> oracle output on rank r's shard."""
    outs = {dt: [shard_step(r, dt, masks_from_numpy(res[r]["masks"])) for r in (0, 1)]
            for dt in (torch.float64, torch.float32)}
    if precision == "bf16":  # the bf16 bars (tests/test_gpu_bf16.py _check_bf16_pinned: the fp32 floor)
        from test_gpu_bf16 import _check_bf16_pinned

        mean = {dt: {k: (o[0]["grads"][k] + o[1]["grads"][k]).detach() / 2 for k in o[0]["grads"]}
                for dt, o in outs.items()}
        _check_bf16_pinned({k: torch.tensor(v) for k, v in res[0]["grad"].items()}, mean[torch.float64],
                           mean[torch.float32], arch, "DP world 2")
        return
    med_tol, worst_tol = PIN[precision]
    rels, over = [], []
    for k, g in res[0]["grad"].items():
        if _bias_before_bn(k, arch):
            continue
        ref = (outs[torch.float64][0]["grads"][k] + outs[torch.float64][1]["grads"][k]).detach() / 2
        f32 = (outs[torch.float32][0]["grads"][k] + outs[torch.float32][1]["grads"][k]).detach().double() / 2
        r, floor = _rel(g, ref), _rel(f32, ref)
        rels.append((r, k, floor))
        if r >= max(worst_tol, FLOOR_X * floor):
            over.append((k, r, floor))
    rels.sort()
    med = rels[len(rels) // 2][0]
    print(f"\npinned DP grads ({precision}): median {med:.2e}; worst (rel, tensor, fp32 floor): "
          + ", ".join(f"({r:.1e}, {k}, {f:.1e})" for r, k, f in rels[-3:]))
    assert med < med_tol, (med, rels[-3:])
    assert not over, over


def _common_checks(res, sd, world=2):
    # construction: every rank holds rank 0's weights
    for k, v in res[0]["p0"].items():
        assert np.array_equal(v, res[1]["p0"][k]), k
        assert np.allclose(v, np.asarray(sd[k], dtype=np.float32), rtol=0, atol=0), k
    # identical parameters after the DP Adam step and after two graph-replayed steps
    for k in res[0]["p1"]:
        assert np.array_equal(res[0]["p1"][k], res[1]["p1"][k]), k
        assert np.array_equal(res[0]["grad"][k], res[1]["grad"][k]), k
    assert np.array_equal(res[0]["p3"], res[1]["p3"])
    assert res[0]["graphs"] and res[1]["graphs"], "DP segments were not graph-captured"
    assert res[0]["opt_step"] == res[1]["opt_step"] == 3
    if "eps" in res[0]:  # each rank draws its own noise stream
        a, b = res[0]["eps"], res[1]["eps"]
        m = min(len(a), len(b))
        assert not np.allclose(a[:m], b[:m], atol=1e-3)


DP_CLEAR = [("VAE", 64, "fp32"), ("VAE", 50, "fp32"),
            # configs[3]'s per-rank shard (PACS: VAE64, 32 per GPU, fp32) and a bf16 VAE64 step (configs[4]'s
            # arithmetic at a small shard)
            ("VAE64", 64, "fp32"), ("VAE64", 32, "bf16")]


@pytest.mark.parametrize("arch,n_global,precision", DP_CLEAR, ids=lambda v: str(v))
def test_dp_clear_step_world2(arch, n_global, precision):
    from oracle import cpu_ref as R
    from test_gpu_bf16 import LOSS_TOL_BF16

    zt, C = (16, 1) if arch == "VAE" else (64, 3)
    res = _launch("clear", n_global, arch=arch, precision=precision, timeout=240 if arch == "VAE64" else 100)
    sd = R.det_state(arch, zt, C)
    _common_checks(res, sd)
    hp = {"temperature": 0.1, "alpha": 100.0, "beta": 0.125, "ps": True}
    x, label, ec, es, _ = R.det_inputs(n_global, C, R.IMAGE[arch], zt, 4, seed=21)
    shards = []
    tol = LOSS_TOL if precision == "fp32" else LOSS_TOL_BF16
    for r in (0, 1):
        lo, hi = res[r]["bounds"]
        o = R.clear_step(R.to_torch(sd), torch.tensor(x[lo:hi]), torch.tensor(label[lo:hi]), torch.tensor(ec[lo:hi]),
                         torch.tensor(es[lo:hi]), arch, hp)
        shards.append(o)
        got = res[r]["losses"]
        for i, k in enumerate(("rec", "kl_c", "kl_s", "c_loss", "s_loss")):
            ref = float(o[k])
            assert abs(float(got[i]) - ref) <= tol * max(abs(ref), 1e-3), (r, k, float(got[i]), ref)
    mean_g = {k: (shards[0]["grads"][k] + shards[1]["grads"][k]) / 2 for k in shards[0]["grads"]}

    def shard_step(r, dt, masks):
        lo, hi = res[r]["bounds"]
        return R.clear_step(R.to_torch(sd, dt), torch.tensor(x[lo:hi], dtype=dt), torch.tensor(label[lo:hi]),
                            torch.tensor(ec[lo:hi], dtype=dt), torch.tensor(es[lo:hi], dtype=dt), arch, hp,
                            masks=masks, bf16=precision == "bf16")

    _check_pinned(res, shard_step, arch, precision)
    if precision == "fp32":
        ref_p = _adam_ref(sd, mean_g, arch=arch)
        prel = sorted((_rel(res[0]["p1"][k], ref_p[k]), k) for k in ref_p)
        assert prel[len(prel) // 2][0] < 1e-5, prel[-3:]
        assert prel[-1][0] < 5e-3, prel[-3:]


@pytest.mark.parametrize("kind,arch", [("CLUBSample", "VAE"), ("L1OutUB", "VAE"), ("CLUBSample", "VAE64")])
def test_dp_mim_step_world2(kind, arch):
    """CLEAR-MIM; the VAE64 case is configs[2]'s model and estimator (CelebA 64x64, CLUB-S) at world 2."""
    from oracle import cpu_ref as R

    n_global = 64 if arch == "VAE" else 32
    zt, C = (16, 1) if arch == "VAE" else (64, 3)
    res = _launch("mim", n_global, kind, arch=arch, timeout=240 if arch == "VAE64" else 100)
    sd = R.det_state(arch, zt, C)
    _common_checks(res, sd)
    for key in ("e0", "e1", "e3"):
        assert np.array_equal(res[0][key], res[1][key]), key
    hp = {"temperature": 0.1, "beta": 0.125, "loc": 0, "scale": 1, "alpha": 100.0, "lambda": 3.0}
    x, label, ec, es, _ = R.det_inputs(n_global, C, R.IMAGE[arch], zt, 4, seed=21)
    gen = np.random.default_rng(5)
    noises = [(ec, es)] + [(gen.standard_normal((n_global, zt // 2)), gen.standard_normal((n_global, zt // 2)))
                           for _ in range(5)]
    M0 = R.to_torch(R.det_mlp(zt // 2, zt))
    shards = []
    for r in (0, 1):
        lo, hi = res[r]["bounds"]
        o = R.mim_step(R.to_torch(sd), M0, torch.tensor(x[lo:hi]), torch.tensor(label[lo:hi]), torch.tensor(ec[lo:hi]),
                       torch.tensor(es[lo:hi]), torch.tensor(res[r]["perm"]), arch, hp, kind)
        shards.append(o)
        got = res[r]["losses"]
        for i, k in ((0, "rec"), (1, "kl_c"), (2, "kl_s"), (3, "c_loss"), (5, "mi")):
            ref = float(o[k])
            assert abs(float(got[i]) - ref) <= LOSS_TOL * max(abs(ref), 1e-2), (r, k, float(got[i]), ref)
    mean_g = {k: (shards[0]["grads"][k] + shards[1]["grads"][k]) / 2 for k in shards[0]["grads"]}

    def shard_step(r, dt, masks):
        lo, hi = res[r]["bounds"]
        return R.mim_step(R.to_torch(sd, dt), R.to_torch(R.det_mlp(zt // 2, zt), dt), torch.tensor(x[lo:hi], dtype=dt),
                          torch.tensor(label[lo:hi]), torch.tensor(ec[lo:hi], dtype=dt), torch.tensor(es[lo:hi], dtype=dt),
                          torch.tensor(res[r]["perm"]), arch, hp, kind, masks=masks)

    _check_pinned(res, shard_step, arch)
    # the estimator: 5 x (per-shard train-mode forward with noise j on the updated VAE, per-shard
    # learning-loss gradient, mean over shards, torch Adam)
    P1 = R.to_torch(sd, requires_grad=False)
    P1.update(_adam_ref(sd, mean_g, arch=arch))
    Ps = [dict(P1), dict(P1)]
    for P in Ps:  # each rank's BN buffers evolve on its own shard
        for k in list(P):
            if "running" in k or "num_batches" in k:
                P[k] = P[k].clone()
    mparams = [M0[k].detach().clone().requires_grad_(True) for k in M0]
    Md = dict(zip(M0.keys(), mparams))
    eopt = torch.optim.Adam(mparams, lr=2e-3)
    for j in range(5):
        a, b = noises[1 + j]
        lls = []
        grads = None
        for r in (0, 1):
            lo, hi = res[r]["bounds"]
            with torch.no_grad():
                _, _, zz = R.vae_forward(Ps[r], torch.tensor(x[lo:hi]), torch.tensor(a[lo:hi]), torch.tensor(b[lo:hi]),
                                         arch, True)
            ll = R.learning_loss(Md, zz[:, : zt // 2], zz[:, zt // 2:])
            g = torch.autograd.grad(ll, mparams)
            grads = [gi / 2 for gi in g] if grads is None else [acc + gi / 2 for acc, gi in zip(grads, g)]
            lls.append(float(ll))
            assert abs(float(res[r]["learn"][j]) - lls[-1]) <= 1e-4 * max(abs(lls[-1]), 1.0), (r, j)
        for p_, g in zip(mparams, grads):
            p_.grad = g
        eopt.step()
    # the estimator arena holds the parameters in est_params order (p_mu then p_logvar, weight, bias)
    ref_e = torch.cat([Md[k].detach().reshape(-1) for k in ("p_mu.0.weight", "p_mu.0.bias", "p_mu.2.weight",
                                                            "p_mu.2.bias", "p_logvar.0.weight", "p_logvar.0.bias",
                                                            "p_logvar.2.weight", "p_logvar.2.bias")])
    e1 = res[0]["e1"]
    got_e = []
    o = 0
    for k in ("p_mu.0.weight", "p_mu.0.bias", "p_mu.2.weight", "p_mu.2.bias", "p_logvar.0.weight", "p_logvar.0.bias",
              "p_logvar.2.weight", "p_logvar.2.bias"):
        nel = Md[k].numel()
        got_e.append(torch.tensor(e1[o:o + nel]))
        o = (o + nel + 3) & ~3
    # 5 Adam steps (lr 2e-3) on gradients that match at ~1e-4: an element whose gradient is near zero can take
    # a +-lr step either way (Adam's first steps are ~lr * sign(g)), so the bar is on Adam's scale: every
    # element within 5 x 2 lr, and rel-L2 1e-3 (VAE, 288 parameters) / 3e-3 (VAE64, 4224 parameters)
    got_e = torch.cat(got_e)
    assert float((got_e.double() - ref_e.double()).abs().max()) <= 10 * 2e-3
    assert _rel(got_e, ref_e) < (1e-3 if arch == "VAE" else 3e-3)


@pytest.mark.parametrize("kind", ["GVAE", "MLVAE"])
def test_dp_group_step_world2(kind):
    from oracle import cpu_ref as R

    n_global, zt = 64, 16
    res = _launch("group", n_global, kind)
    sd = R.det_state("VAE", zt, 1)
    _common_checks(res, sd)
    hp = {"beta": 0.125, "loc": 0, "scale": 1}
    x, label, ec, es, _ = R.det_inputs(n_global, 1, 28, zt, 4, seed=21)
    shards = []
    for r in (0, 1):
        lo, hi = res[r]["bounds"]
        o = R.group_step(R.to_torch(sd), torch.tensor(x[lo:hi]), torch.tensor(label[lo:hi]),
                         R.group_order_noise(label[lo:hi], torch.tensor(ec[lo:hi])), torch.tensor(es[lo:hi]), "VAE",
                         hp, kind)
        shards.append(o)
        got = res[r]["losses"]
        for i, k in ((0, "rec_adj"), (1, "kl_c"), (2, "kl_s_adj")):
            ref = float(o[k])
            assert abs(float(got[i]) - ref) <= LOSS_TOL * max(abs(ref), 1e-3), (r, k, float(got[i]), ref)
    mean_g = {k: (shards[0]["grads"][k] + shards[1]["grads"][k]) / 2 for k in shards[0]["grads"]}

    def shard_step(r, dt, masks):
        lo, hi = res[r]["bounds"]
        return R.group_step(R.to_torch(sd, dt), torch.tensor(x[lo:hi], dtype=dt), torch.tensor(label[lo:hi]),
                            R.group_order_noise(label[lo:hi], torch.tensor(ec[lo:hi], dtype=dt)),
                            torch.tensor(es[lo:hi], dtype=dt), "VAE", hp, kind, masks=masks)

    _check_pinned(res, shard_step, "VAE")
    ref_p = _adam_ref(sd, mean_g)
    prel = sorted((_rel(res[0]["p1"][k], ref_p[k]), k) for k in ref_p)
    assert prel[len(prel) // 2][0] < 1e-5, prel[-3:]
    assert prel[-1][0] < 5e-3, prel[-3:]


def test_dp_tc_step_world2():
    from oracle import cpu_ref as R

    n_global, zt = 64, 16
    res = _launch("tc", n_global)
    sd = R.det_state("VAE", zt, 1)
    _common_checks(res, sd)
    for key in ("e0", "e1", "e3"):
        assert np.array_equal(res[0][key], res[1][key]), key
    hp = {"temperature": 0.1, "beta": 0.125, "loc": 0, "scale": 1, "alpha": 100.0, "lambda": 3.0}
    x, label, ec, es, _ = R.det_inputs(n_global, 1, 28, zt, 4, seed=21)
    gen = np.random.default_rng(6)
    a2, b2 = gen.standard_normal((n_global, zt // 2)), gen.standard_normal((n_global, zt // 2))
    D0 = R.to_torch(R.det_disc(zt))
    shards = []
    for r in (0, 1):
        lo, hi = res[r]["bounds"]
        o = R.tc_step(R.to_torch(sd), D0, torch.tensor(x[lo:hi]), torch.tensor(label[lo:hi]), torch.tensor(ec[lo:hi]),
                      torch.tensor(es[lo:hi]), "VAE", hp)
        shards.append(o)
        got = res[r]["losses"]
        for i, k in ((0, "rec"), (1, "kl_c"), (2, "kl_s"), (3, "c_loss")):
            ref = float(o[k].detach())
            assert abs(float(got[i]) - ref) <= LOSS_TOL * max(abs(ref), 1e-3), (r, k, float(got[i]), ref)
        mi = float(o["mi"].detach())
        assert abs(float(got[5]) - mi) <= LOSS_TOL * max(abs(mi), 1.0), (r, float(got[5]), mi)
    mean_g = {k: (shards[0]["grads"][k] + shards[1]["grads"][k]) / 2 for k in shards[0]["grads"]}

    def shard_step(r, dt, masks):
        lo, hi = res[r]["bounds"]
        return R.tc_step(R.to_torch(sd, dt), R.to_torch(R.det_disc(zt), dt), torch.tensor(x[lo:hi], dtype=dt),
                         torch.tensor(label[lo:hi]), torch.tensor(ec[lo:hi], dtype=dt), torch.tensor(es[lo:hi], dtype=dt),
                         "VAE", hp, masks=masks)

    _check_pinned(res, shard_step, "VAE")
    # the discriminator step: per-shard BCE on z of the second forward (fresh noise, post-Adam VAE), gradients
    # averaged over the shards, torch Adam
    P1 = R.to_torch(sd, requires_grad=False)
    P1.update(_adam_ref(sd, mean_g))
    Dp = [v.detach().clone().requires_grad_(True) for v in D0.values()]
    Dd = dict(zip(D0.keys(), Dp))
    grads = None
    for r in (0, 1):
        lo, hi = res[r]["bounds"]
        P = {k: (v.clone() if ("running" in k or "num_batches" in k) else v) for k, v in P1.items()}
        with torch.no_grad():
            _, _, z2 = R.vae_forward(P, torch.tensor(x[lo:hi]), torch.tensor(a2[lo:hi]), torch.tensor(b2[lo:hi]),
                                     "VAE", True)
        fl = R.tc_factor_loss(Dd, z2)
        assert abs(float(res[r]["learn"][0]) - float(fl)) <= 1e-3 * abs(float(fl)), (r, float(res[r]["learn"][0]))
        g = torch.autograd.grad(fl, Dp)
        grads = [gi / 2 for gi in g] if grads is None else [acc + gi / 2 for acc, gi in zip(grads, g)]
    for p_, g in zip(Dp, grads):
        p_.grad = g
    torch.optim.Adam(Dp, lr=1e-3).step()
    ref_e = torch.cat([Dd[k].detach().reshape(-1) for k in ("0.weight", "0.bias", "2.weight", "2.bias")])
    e1, got_e, o = res[0]["e1"], [], 0
    for k in ("0.weight", "0.bias", "2.weight", "2.bias"):
        nel = Dd[k].numel()
        got_e.append(torch.tensor(e1[o:o + nel]))
        o = (o + nel + 3) & ~3
    assert _rel(torch.cat(got_e), ref_e) < 1e-3
