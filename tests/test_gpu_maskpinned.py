"""Gradient parity with the ReLU activity pinned: the fused step's gradients against the fp64 oracle run
with the ReLU masks the HIP forward actually chose.

test_gpu_golden.py / test_gpu_parity.py have to hold gradients at a per-tensor bar of 2e-2: a ReLU whose
BatchNorm output is within fp32 rounding of 0 can take the other branch than in fp64, and that one
element's changed gradient spreads upstream at ~1e-3 (DESIGN.md "Numerics").  Here the oracle
(oracle/cpu_ref.py, `masks=`) evaluates every BN -> ReLU of the encoder and decoder as h * mask with the
device's own masks, so the comparison is between two evaluations of the same smooth function: every
gradient tensor is then held at the fp32-accumulation floor (bars below), which would expose a wrong
BatchNorm-affine, bias or weight-gradient kernel on any tensor, however small.

Device masks: the forward stores pre-BN activations (NHWC); the mask of layer l is BN_l(y_l) > 0 evaluated
by cv_bn_apply with the step's own batch statistics — the arithmetic of the GEMM prologues' BN+ReLU
transform (bn_out in cv_common.hpp, fmaf((x - mu), sc, beta)); the BatchNorm1d's mask is its stored
output ah > 0.  The step is run as its programs up to the end of the backward (forward, decoder backward,
latent terms, encoder backward + reduction), before Adam moves the weights.  The estimators' and the
factor discriminator's own hidden ReLUs are not pinned (64-1024 elements; no flip in these cases).

Reference step: /root/reference/code/src/trainer.py:452-482 (CLEAR), :848-869 (CLEAR-MIM), :654-677
(CLEAR-TC), :335-353 (GVAE / ML-VAE)."""

import numpy as np
import pytest
import torch

import golden_cases as G
from maskpin import device_masks
from test_gpu_golden import _bias_before_bn, build_fused

pytestmark = pytest.mark.gpu

# rel-L2 per gradient tensor against the fp64 pinned oracle: the median tensor, and every tensor at
# max(WORST_TOL, FLOOR_X x the fp32 floor of that tensor).  The fp32 floor is the same pinned oracle run in
# fp32 on the host: a tensor that is a cancelling sum over the batch (a head bias: sum_n d(head)) carries
# a relative error far above 1e-5 in ANY fp32 evaluation (measured up to 2e-4), so its bar is set by the
# fp32 arithmetic itself, not by a fixed number.
MEDIAN_TOL = 5e-6
WORST_TOL = 1e-5
FLOOR_X = 8.0


def oracle_grads(fx, masks, dtype=torch.float64):
    from oracle import cpu_ref as R

    m = fx["meta"]
    arch, mode = m["arch"], m["mode"]
    x, label, ec, es, perm = G.inputs(fx)
    hp = G.hyper(fx)
    P = R.to_torch(R.det_state(arch, m["z"], m["C"]), dtype)
    X, L = torch.tensor(x, dtype=dtype), torch.tensor(label)
    Ec, Es = torch.tensor(ec, dtype=dtype), torch.tensor(es, dtype=dtype)
    if mode == "group":
        o = R.group_step(P, X, L, R.group_order_noise(label, Ec), Es, arch, hp, m["estimator"], masks=masks)
    elif mode == "clear":
        o = R.clear_step(P, X, L, Ec, Es, arch, hp, m["sim_fn"], masks=masks)
    elif mode == "tc":
        o = R.tc_step(P, R.to_torch(R.det_disc(m["z"]), dtype), X, L, Ec, Es, arch, hp, m["sim_fn"], masks=masks)
    else:
        o = R.mim_step(P, R.to_torch(R.det_mlp(m["z"] // 2, m["z"]), dtype), X, L, Ec, Es, torch.tensor(perm), arch, hp,
                       m["estimator"], m["sim_fn"], masks=masks)
    return o


@pytest.mark.parametrize("name", G.names())
def test_fused_grads_mask_pinned(name):
    from cvhip import _lib

    fx = G.load(name)
    m = fx["meta"]
    arch = m["arch"]
    x, label, _, _, _ = G.inputs(fx)
    tr, eng, _ = build_fused(fx)
    n = x.shape[0]
    Gp = eng._programs(n)
    eng._load_batch(Gp, torch.tensor(x, dtype=torch.float32, device="cuda"), torch.tensor(label, device="cuda"))
    assert eng._take_injections(Gp)
    s = _lib.stream_handle()
    for P in (Gp["fwd_inj"], Gp["dec"], Gp["lat_inj"], Gp["enc"]):
        P.run(s)
    torch.cuda.synchronize()
    masks = device_masks(eng, Gp["ws"], n)
    o = oracle_grads(fx, masks)
    o32 = oracle_grads(fx, masks, torch.float32)
    rels, over = [], []
    for k, p in tr.model.named_parameters():
        g_ref = o["grads"][k].detach()
        g = p.grad.detach().double().cpu()
        if _bias_before_bn(k, arch):
            assert float(g.abs().max()) == 0.0, k
            continue
        r = G.rel(g.numpy(), g_ref.numpy())
        floor = G.rel(o32["grads"][k].detach().double().numpy(), g_ref.numpy())
        rels.append((r, k, floor))
        if r >= max(WORST_TOL, FLOOR_X * floor):
            over.append((k, r, floor))
    rels.sort()
    med = rels[len(rels) // 2][0]
    print(f"\n{name}: median {med:.2e}; worst (rel, tensor, fp32 floor): "
          + ", ".join(f"({r:.1e}, {k}, {f:.1e})" for r, k, f in rels[-3:]))
    assert med < MEDIAN_TOL, (med, rels[-3:])
    assert not over, over
