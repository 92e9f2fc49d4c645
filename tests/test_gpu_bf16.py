"""bf16 MFMA path (BASELINE configs[4]: "Camelyon17 ... bs=1024 bf16", cvhip.plan.set_precision) against the
fp64 oracle on identical weights, inputs and noise.

The reference computes in fp32 only; with precision="bf16" the conv / linear contractions of the GEMM core
take bf16-rounded operands (8-bit mantissa, unit roundoff 2^-9 = 2.0e-3) with fp32 accumulation, while the
image-facing edge layers, BatchNorm statistics, the ELBO / contrastive reductions and Adam stay fp32.  The
tolerances below are stated for that arithmetic (a bf16 product carries up to ~4e-3 relative error; the
BatchNorm after every conv renormalises, so the errors do not compound with depth):

  * losses (rec, KL_c, KL_s, contrastive): 1e-2 relative (the reduction over N*C*H*W or N*d elements
    averages the per-element rounding);
  * encoded latents (mu / logvar heads, z) and x_hat: 3e-2 relative L2;
  * gradients against the plain fp64 oracle: whole-model relative L2 < 0.15 and median per-tensor < 0.15
    (measured 0.04-0.09 at N=32..128: at initialisation many BatchNorm outputs sit near 0, and a bf16 forward
    flips the ReLU of ~0.1% of them against fp64, each flip changing that element's whole upstream gradient);
    test_bf16_step_mask_pinned removes the ReLU flips (the device's pattern pinned) and restates the bf16
    rounding in the oracle, and holds every tensor to the fp32 floor of that function (_check_bf16_pinned);
  * the same step in fp32 on the same engine stays within the fp32 bar (1e-4), so the looser numbers
    are the bf16 operands' and nothing else;
  * kernel level (below): with bf16-representable operands the bf16 core matches an fp64 contraction at
    1e-5, the fp32 kernels' bar, so the rounding points are the only difference.
"""

import numpy as np
import pytest
import torch

from test_gpu_parity import _bias_before_bn, _fused_trainer, _rel

pytestmark = pytest.mark.gpu

LOSS_TOL_BF16 = 1e-2
LATENT_TOL_BF16 = 3e-2
GRAD_TOL_BF16 = 0.15


def _step(arch, zt, C, n, precision, sd, x, label, ec, es, hp):
    from cvhip import rng
    from cvhip.engine import ClearStep
    from cvhip.plan import set_precision

    tr = _fused_trainer(arch, zt, C, sd, hp, lr=3e-5)
    set_precision(tr.model, precision)
    eng = ClearStep.build(tr, "clear")
    assert eng is not None and eng.spec.mma == (1 if precision == "bf16" else 0)
    rng.clear_injections()
    rng.inject_noise([torch.tensor(ec, dtype=torch.float32), torch.tensor(es, dtype=torch.float32)])
    losses = eng.step(torch.tensor(x, dtype=torch.float32, device="cuda"), torch.tensor(label, device="cuda"))
    torch.cuda.synchronize()
    ws = eng.last_workspace(n)
    grads = {k: p.grad.detach().clone() for k, p in tr.model.named_parameters()}
    return losses.clone().cpu(), ws.heads.clone().cpu(), ws.z.clone().cpu(), grads, eng


@pytest.mark.parametrize("arch,zt,C,n", [("VAE64", 64, 3, 32), ("VAE64", 64, 3, 128), ("VAE", 16, 1, 128)])
def test_bf16_fused_step_vs_oracle(arch, zt, C, n):
    from oracle import cpu_ref as R

    sd = R.det_state(arch, zt, C)
    x, label, ec, es, _ = R.det_inputs(n, C, R.IMAGE[arch], zt, 2)
    hp = {"temperature": 0.1, "alpha": 100.0, "beta": 1 / 32, "ps": True, "loc": 0, "scale": 1}
    o = R.clear_step(R.to_torch(sd), torch.tensor(x), torch.tensor(label), torch.tensor(ec), torch.tensor(es), arch,
                     hp)
    d = zt // 2
    ref_heads = torch.cat([o[k] for k in ("mu_c", "logvar_c", "mu_s", "logvar_s")], dim=1)
    errs = {}
    for precision in ("fp32", "bf16"):
        losses, heads, z, grads, eng = _step(arch, zt, C, n, precision, sd, x, label, ec, es, hp)
        e = {}
        for i, k in enumerate(("rec", "kl_c", "kl_s", "c_loss", "s_loss")):
            ref = float(o[k])
            e[k] = abs(float(losses[i]) - ref) / max(abs(ref), 1e-3)
        e["heads"] = _rel(heads, ref_heads)
        e["z"] = _rel(z, o["z"])
        num = den = 0.0
        per = []
        for k, g_ref in o["grads"].items():
            if _bias_before_bn(k, arch):
                continue
            g = grads[k].double().cpu()
            num += float((g - g_ref.double()).norm() ** 2)
            den += float(g_ref.double().norm() ** 2)
            per.append(_rel(g, g_ref))
        e["grad_global"] = (num / den) ** 0.5
        e["grad_median"] = sorted(per)[len(per) // 2]
        errs[precision] = e
    print(f"\n{arch} n={n} errors:", {p: {k: f"{v:.2e}" for k, v in e.items()} for p, e in errs.items()})
    f, b = errs["fp32"], errs["bf16"]
    for k in ("rec", "kl_c", "kl_s", "c_loss", "s_loss"):
        assert f[k] < 1e-4, ("fp32", k, f[k])
        assert b[k] < LOSS_TOL_BF16, ("bf16", k, b[k])
    for k in ("heads", "z"):
        assert f[k] < 2e-5, ("fp32", k, f[k])
        assert b[k] < LATENT_TOL_BF16, ("bf16", k, b[k])
    assert b["grad_global"] < GRAD_TOL_BF16 and b["grad_median"] < GRAD_TOL_BF16, b
    # bf16 is really in effect (not a silent fp32 run): its latents differ from the fp32 run's
    assert b["heads"] > 10 * f["heads"]


@pytest.mark.parametrize("arch,zt,C,n", [("VAE64", 64, 3, 32), ("VAE64", 64, 3, 128), ("VAE", 16, 1, 128)])
def test_bf16_step_mask_pinned(arch, zt, C, n):
    """The bf16 step against the oracle that rounds the same operands to bf16 at the same points
    (oracle/cpu_ref.py `bf16=`: the GEMM-core convs' input activation after its BN+ReLU, the weight, and the
    incoming gradient after the BN backward; fp64 accumulation) with the device's ReLU activity pinned
    (tests/maskpin.py).  What remains is fp32 accumulation order and the rare bf16 tie broken differently by an
    fp32 vs fp64 pre-rounding value, which the function amplifies (_check_bf16_pinned): heads and z within 1e-4
    relative, losses within max(1e-4 relative, 2 x the fp32 oracle's own deviation), gradients at the fp32 floor."""
    from cvhip import rng
    from cvhip.engine import ClearStep
    from cvhip.plan import set_precision
    from maskpin import device_masks
    from oracle import cpu_ref as R

    sd = R.det_state(arch, zt, C)
    x, label, ec, es, _ = R.det_inputs(n, C, R.IMAGE[arch], zt, 2)
    hp = {"temperature": 0.1, "alpha": 100.0, "beta": 1 / 32, "ps": True, "loc": 0, "scale": 1}
    tr = _fused_trainer(arch, zt, C, sd, hp, lr=3e-5)
    set_precision(tr.model, "bf16")
    eng = ClearStep.build(tr, "clear")
    assert eng is not None and eng.spec.mma == 1
    rng.clear_injections()
    rng.inject_noise([torch.tensor(ec, dtype=torch.float32), torch.tensor(es, dtype=torch.float32)])
    held = {}
    losses = eng.step(torch.tensor(x, dtype=torch.float32, device="cuda"), torch.tensor(label, device="cuda"),
                      before_update=lambda: held.update(m=device_masks(eng, eng.last_workspace(n), n)))
    torch.cuda.synchronize()
    ws = eng.last_workspace(n)
    losses, heads, z = losses.cpu(), ws.heads.cpu(), ws.z.cpu()
    grads = {k: p.grad.detach().double().cpu() for k, p in tr.model.named_parameters()}

    def oracle(dt):
        return R.clear_step(R.to_torch(sd, dt), torch.tensor(x, dtype=dt), torch.tensor(label),
                            torch.tensor(ec, dtype=dt), torch.tensor(es, dtype=dt), arch, hp, masks=held["m"], bf16=True)

    o, o32 = oracle(torch.float64), oracle(torch.float32)
    cat = lambda d: torch.cat([d[k] for k in ("mu_c", "logvar_c", "mu_s", "logvar_s")], dim=1).detach()
    ref_heads = cat(o)
    # the forward's own fp32 floor: the fp32 oracle's heads / z against its fp64 evaluation of the same function
    hfloor = _rel(cat(o32).double(), ref_heads)
    zfloor = _rel(o32["z"].detach().double(), o["z"].detach())
    eh, ez = _rel(heads, ref_heads), _rel(z, o["z"].detach())
    print(f"\n{arch} n={n} bf16 pinned forward: heads {eh:.2e} (floor {hfloor:.2e}), z {ez:.2e} (floor {zfloor:.2e})")
    assert eh < max(1e-4, PIN_FLOOR_X * hfloor) and ez < max(1e-4, PIN_FLOOR_X * zfloor), (eh, hfloor, ez, zfloor)
    for i, k in enumerate(("rec", "kl_c", "kl_s", "c_loss", "s_loss")):
        ref = float(o[k])
        # a scalar's fp32 floor is one sample of the rounding noise, so it is floored by the noise its inputs
        # (the heads) carry: a loss is no better pinned than the latents it is computed from
        floor = max(abs(float(o32[k]) - ref), hfloor * abs(ref))
        assert abs(float(losses[i]) - ref) <= max(1e-4 * max(abs(ref), 1e-3), PIN_FLOOR_X * floor), (
            k, float(losses[i]), ref, floor)
    _check_bf16_pinned({k: grads[k] for k in o["grads"]}, o["grads"], o32["grads"], arch, f"{arch} n={n}")


# The bf16-rounding function is ill-conditioned in a way fp32 is not: an operand within fp32 rounding of a bf16
# rounding midpoint rounds either way, each such flip moves that operand by 2^-8, and the flips multiply layer
# after layer.  So even the oracle's own fp32 evaluation of the identical function (same masks, same rounding
# points) lands 1e-3 - 6e-3 from its fp64 evaluation per gradient tensor (measured; the fp32 "floor").  The device
# can be no closer; the bars hold it to that floor: every tensor within max(1e-3, PIN_FLOOR_X x its floor) and the
# median tensor within max(1e-4, PIN_FLOOR_X x the median floor).  (A wrong bf16 weight gradient on any tensor
# is off by O(1), far outside.)  On top, a fixed cap PIN_CAP on every tensor, whatever its floor.  The cap is 1e-2,
# not 5e-3: the floor itself reaches 8.0e-3 (VAE64 n=32 encoder.1.weight; the per-tensor table is in DESIGN.md §2),
# so no fp32 evaluation of this function passes 5e-3 on every tensor.  Measured device / floor ratios are
# 0.5-1.3 (round 5), so PIN_FLOOR_X is 1.5 (was 2).
PIN_FLOOR_X = 1.5
PIN_CAP = 1e-2


def _check_bf16_pinned(got, ref64, ref32, arch, what):
    rels, over = [], []
    for k, g_ref in ref64.items():
        if _bias_before_bn(k, arch):
            continue
        r = _rel(got[k], g_ref.detach())
        floor = _rel(ref32[k].detach().double(), g_ref.detach())
        rels.append((r, k, floor))
        if r >= min(PIN_CAP, max(1e-3, PIN_FLOOR_X * floor)):
            over.append((k, r, floor))
    rels.sort()
    med = rels[len(rels) // 2][0]
    fmed = sorted(f for _, _, f in rels)[len(rels) // 2]
    print(f"\n{what} bf16 pinned: median {med:.2e} (floor median {fmed:.2e}); worst (rel, tensor, fp32 floor): "
          + ", ".join(f"({r:.1e}, {k}, {f:.1e})" for r, k, f in rels[-3:]))
    print(f"{what} per-tensor table (rel, fp32 floor): "
          + "; ".join(f"{k} {r:.2e} {f:.2e}" for r, k, f in sorted(rels, key=lambda v: v[1])))
    assert med < max(1e-4, PIN_FLOOR_X * fmed), (med, fmed, rels[-3:])
    assert not over, over


def test_bf16_training_decreases_loss():
    """Camelyon-shaped VAE64 at bs=128 in bf16 through get_clearvae_trainer(precision="bf16").fit."""
    from oracle import cpu_ref as R
    from src.utils.trainer_utils import get_clearvae_trainer

    torch.manual_seed(0)
    tr = get_clearvae_trainer(beta=1 / 32, ps=True, vae_lr=3e-4, z_dim=64, alpha=100, temperature=0.1,
                              device="cuda", vae_arch="VAE64", in_channel=3, verbose_period=100, precision="bf16")
    x, label, _, _, _ = R.det_inputs(256, 3, 64, 64, 2, seed=9)
    ds = torch.utils.data.TensorDataset(torch.tensor(x, dtype=torch.float32), torch.tensor(label))
    dl = torch.utils.data.DataLoader(ds, batch_size=128, shuffle=False)
    tr.fit(1, dl)
    eng = tr._engine
    assert eng is not None and eng.spec.mma == 1
    first = eng.last_workspace(128).losses.clone()
    tr.fit(6, dl)
    last = eng.last_workspace(128).losses.clone()
    assert torch.isfinite(last[:5]).all()
    assert float(last[0]) < float(first[0])


# ----------------------------------------------------------------------------- kernel level
# With operands that are exactly representable in bf16, the bf16 core's products are exact in fp32, so
# its results must match an fp64 host contraction to fp32-accumulation accuracy (1e-5) - the same bar as
# the fp32 kernels in test_gpu_conv_kernels.py.  With arbitrary fp32 operands the core layers must
# differ from the exact contraction by bf16 rounding (>1e-4), i.e. bf16 really ran; the image-facing
# layers (edge kernels, fp32 by design) must not.

from test_gpu_conv_kernels import GEOMS, _packed, rel  # noqa: E402


def _b16(t):
    return t.to(torch.bfloat16).to(torch.float32)


@pytest.mark.parametrize("geom", GEOMS, ids=lambda g: "T" * g[1] + f"{g[2]}x{g[3]}-{g[4]}x{g[5]}k{g[6]}")
def test_bf16_conv_kernels(geom):
    import torch.nn.functional as F

    from cvhip import _lib

    n, tr, cin, hin, cout, hout, k, s, p = geom
    dev = torch.device("cuda")
    rng = np.random.default_rng(hash(geom) % 2**32)
    op = (hout - ((hin - 1) * s - 2 * p + k)) if tr else 0
    g = _lib.cv_conv(n, cin, hin, hin, cout, hout, hout, k, k, s, p, tr, _lib.MMA_BF16)
    wshape = (cin, cout, k, k) if tr else (cout, cin, k, k)
    edge = cin in (1, 3) or cout in (1, 3)
    s_ = _lib.stream_handle()
    for exact in (True, False):
        W = torch.tensor(rng.uniform(-0.2, 0.2, wshape), dtype=torch.float32, device=dev)
        x = torch.tensor(rng.standard_normal((n, hin, hin, cin)), dtype=torch.float32, device=dev)
        dy = torch.tensor(rng.standard_normal((n, hout, hout, cout)), dtype=torch.float32, device=dev)
        if exact:
            W, x, dy = _b16(W), _b16(x), _b16(dy)
        Wf, Wb = _packed(_lib, W, tr)
        opnd = _lib.cv_operand(x.data_ptr(), None, _lib.XF_NONE, 0)
        gop = _lib.cv_operand(dy.data_ptr(), None, _lib.XF_NONE, 0)
        out = torch.empty(n, hout, hout, cout, dtype=torch.float32, device=dev)
        _lib.call("cv_conv_forward", g, opnd, Wf.data_ptr(), None, out.data_ptr(), _lib.cv_epilogue(), s_)
        gin = torch.empty(n, hin, hin, cin, dtype=torch.float32, device=dev)
        _lib.call("cv_conv_backward_data", g, gop, Wb.data_ptr(), gin.data_ptr(), _lib.cv_epilogue(), s_)
        wb = _lib.lib().cv_conv_wgrad_workspace_bytes(g, 0)
        work = torch.empty(max(wb // 4, 1), dtype=torch.float32, device=dev)
        gw = torch.zeros(wshape, dtype=torch.float32, device=dev)
        _lib.call("cv_conv_backward_weight", g, opnd, gop, gw.data_ptr(), None, 0, work.data_ptr(), wb, s_)
        torch.cuda.synchronize()
        xd, Wd, dyd = (t.double().cpu() for t in (x.permute(0, 3, 1, 2), W, dy.permute(0, 3, 1, 2)))
        if tr:
            ref = F.conv_transpose2d(xd, Wd, None, stride=s, padding=p, output_padding=op)
            gref = F.conv2d(dyd, Wd, None, stride=s, padding=p)
            wref = torch.nn.grad.conv2d_weight(dyd, (cin, cout, k, k), xd, stride=s, padding=p)
        else:
            ref = F.conv2d(xd, Wd, None, stride=s, padding=p)
            gref = torch.nn.grad.conv2d_input((n, cin, hin, hin), Wd, dyd, stride=s, padding=p)
            wref = torch.nn.grad.conv2d_weight(xd, wshape, dyd, stride=s, padding=p)
        errs = (rel(out, ref.permute(0, 2, 3, 1)), rel(gin, gref.permute(0, 2, 3, 1)), rel(gw, wref))
        if exact:
            assert max(errs) < 1e-5, ("bf16-exact operands", errs)
        elif not edge:
            assert min(errs) > 1e-4, ("bf16 rounding not in effect", errs)
            assert max(errs) < 2e-2, ("bf16 error too large", errs)


def test_bf16_linear_heads():
    """cv_linear_forward / backward_data in bf16 on the VAE64 heads shape (DENSE core)."""
    from cvhip import _lib

    dev = torch.device("cuda")
    rng = np.random.default_rng(3)
    n, fin, fout = 64, 2048, 128
    g = _lib.cv_linear(n, fin, fout, 1, 0, 1, 0, _lib.MMA_BF16)
    x = _b16(torch.tensor(rng.standard_normal((n, fin)), dtype=torch.float32, device=dev))
    W = _b16(torch.tensor(rng.uniform(-0.05, 0.05, (fout, fin)), dtype=torch.float32, device=dev))
    dy = _b16(torch.tensor(rng.standard_normal((n, fout)), dtype=torch.float32, device=dev))
    out = torch.empty(n, fout, device=dev)
    _lib.call("cv_linear_forward", g, _lib.cv_operand(x.data_ptr(), None, 0, 0), W.data_ptr(), None,
              out.data_ptr(), 0, _lib.cv_epilogue(), _lib.stream_handle())
    gin = torch.empty(n, fin, device=dev)
    _lib.call("cv_linear_backward_data", g, _lib.cv_operand(dy.data_ptr(), None, 0, 0), W.data_ptr(),
              gin.data_ptr(), 0, _lib.cv_epilogue(), _lib.stream_handle())
    torch.cuda.synchronize()
    assert rel(out, x.double() @ W.double().T) < 1e-5
    assert rel(gin, dy.double() @ W.double()) < 1e-5
