"""NT-Xent phases in the decoder-input launches (cvhip/engine.py LATENT_AUX_DL, csrc/cv_declinear.hip
declinear_{fwd,bwd}_aux_kernel): the row log-sum-exps ride in the decoder-input forward's grid, the losses and
gradients in the decoder-input backward's.  Reference terms: trainer.py:474-479 via losses.py:98-137.

For MNIST's VAE (d = 8, n = 512) and VAE64 (d = 32, n = 64 and the C3 / CelebA batch n = 256), one fused CLEAR step
with injected noise, the phases in the decoder-input grids against the previous placement (the decoder
ConvTranspose2d grids, or their own launches where those do not serve the phase):
  * the two phases really merged into the decoder-input launches (cv_debug_aux_count: 2 per step);
  * heads, d(heads), losses and every gradient agree to 1e-6 relative (the same NT-Xent bodies on the same data;
    d(heads) takes the same adds in the same order), and the losses match the fp64 oracle at the parity bar."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(dl, arch, zt, C, hw, n):
    from oracle import cpu_ref as R
    from cvhip import _lib, engine, rng
    from cvhip.engine import ClearStep
    from test_gpu_parity import _fused_trainer

    L = _lib.lib()
    prev = engine.LATENT_AUX_DL
    engine.LATENT_AUX_DL = 2 if dl else 0  # (2: also where the ConvTranspose2d grids would serve the phase)
    try:
        sd = R.det_state(arch, zt, C)
        x, label, ec, es, _ = R.det_inputs(n, C, hw, zt, 4)
        hp = {"temperature": 0.1, "alpha": 100.0, "beta": 0.125, "ps": True, "loc": 0, "scale": 1}
        tr = _fused_trainer(arch, zt, C, sd, hp)
        eng = ClearStep.build(tr, "clear")
        rng.clear_injections()
        rng.inject_noise([torch.tensor(ec, dtype=torch.float32), torch.tensor(es, dtype=torch.float32)])
        L.cv_debug_aux_count(1)
        held = {}

        def grab():
            ws = eng.last_workspace(n)
            held.update(heads=ws.heads.clone().cpu(), dheads=ws.dheads.clone().cpu(),
                        grads={k: p.grad.detach().clone().cpu() for k, p in tr.model.named_parameters()})

        losses = eng.step(torch.tensor(x, dtype=torch.float32, device="cuda"), torch.tensor(label, device="cuda"),
                          before_update=grab).clone().cpu()
        torch.cuda.synchronize()
        merged = L.cv_debug_aux_count(1)
        names = [c[0] for c in eng.graphs[n]["dec"].calls]
    finally:
        engine.LATENT_AUX_DL = prev
    return dict(losses=losses, merged=merged, names=names, **held), (x, label, ec, es, hp, sd)


def _rel(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("arch,zt,C,hw,n", [("VAE", 16, 1, 28, 512), ("VAE64", 64, 3, 64, 64),
                                            ("VAE64", 64, 3, 64, 256)])
def test_phases_in_decoder_input_launches(arch, zt, C, hw, n):
    from oracle import cpu_ref as R

    new, inp = _run(True, arch, zt, C, hw, n)
    old, _ = _run(False, arch, zt, C, hw, n)
    assert new["merged"] == 2, new["merged"]
    assert "cv_ntxent_aux" in new["names"] and "cv_ntxent_aux" not in old["names"]
    for k in ("heads", "dheads"):
        assert _rel(new[k], old[k]) < 1e-6, (k, _rel(new[k], old[k]))
    assert _rel(new["losses"][:5], old["losses"][:5]) < 1e-6, (new["losses"][:5], old["losses"][:5])
    worst = max(_rel(new["grads"][k], old["grads"][k]) for k in old["grads"] if float(old["grads"][k].norm()) > 0)
    assert worst < 1e-5, worst
    x, label, ec, es, hp, sd = inp
    o = R.clear_step(R.to_torch(sd), torch.tensor(x), torch.tensor(label), torch.tensor(ec), torch.tensor(es), arch,
                     hp)
    for i, k in enumerate(("rec", "kl_c", "kl_s", "c_loss", "s_loss")):
        ref = float(o[k])
        assert abs(float(new["losses"][i]) - ref) <= 1e-4 * max(abs(ref), 1e-3), (k, float(new["losses"][i]), ref)
