"""NT-Xent phases inside the decoder forward (csrc/cv_aux.hip, cvhip/engine.py LATENT_AUX): the row log-sum-exps ride
as extra workgroups of the first decoder ConvTranspose2d's direct launch, the losses and gradients (accumulated into
the zeroed d(heads)) in the second's, and the KL / decoder-chain seed adds onto them after the decoder backward
(reference: trainer.py:474-479 via losses.py:98-137 for the contrastive terms, trainer.py:476-477 for the KL).

The MNIST-shaped fused CLEAR step (VAE z = 16, n = 512, injected noise) runs with the phases merged (default) and
with the previous schedule (cv_latent_step after the decoder backward):
  * the merged grids really ran (cv_debug_aux_count: 2 per step) and not in the old schedule;
  * losses, heads, d(heads) and every gradient agree to 1e-6 relative (the same kernels; d(heads) gets the same two
    adds per element in the other order; the remaining run-to-run spread is the fp32-atomic dz partials);
  * both match the fp64 oracle at the parity bar (1e-4 on the losses).
Also with the merge switched off in the library (cv_debug_aux(0)): the queued phases launch on their own at the
flush points, same results.  Both with the combine split (LATENT_CHAIN, opt-in — measured slower, engine.py keeps it
off: its KL part rides in the rows-phase grid, the decoder-chain part in the heads backward — d(heads) in memory then lacks the chain term, which the test
adds from z / dz / heads) and with the one-launch combine after the decoder backward; and with the gradient phase
queued before the output-loss launch instead (LATENT_AUX_OUT, cv_output_loss serves it)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N = 512


def _run(aux_engine, aux_lib, chain=True):
    from oracle import cpu_ref as R
    from cvhip import _lib, engine, rng
    from cvhip.engine import ClearStep
    from test_gpu_parity import _fused_trainer

    L = _lib.lib()
    prev_e, prev_l, prev_c = engine.LATENT_AUX, L.cv_debug_aux(1 if aux_lib else 0), engine.LATENT_CHAIN
    engine.LATENT_AUX = aux_engine
    engine.LATENT_CHAIN = chain
    try:
        sd = R.det_state("VAE", 16, 1)
        x, label, ec, es, _ = R.det_inputs(N, 1, 28, 16, 10)
        hp = {"temperature": 0.1, "alpha": 100.0, "beta": 0.125, "ps": True, "loc": 0, "scale": 1}
        tr = _fused_trainer("VAE", 16, 1, sd, hp)
        eng = ClearStep.build(tr, "clear")
        rng.clear_injections()
        rng.inject_noise([torch.tensor(ec, dtype=torch.float32), torch.tensor(es, dtype=torch.float32)])
        L.cv_debug_aux_count(1)
        held = {}

        def grab():
            ws = eng.last_workspace(N)
            held.update(heads=ws.heads.clone().cpu(), dheads=ws.dheads.clone().cpu(), z=ws.z.clone().cpu(),
                        dz=ws.dz.clone().cpu(),
                        grads={k: p.grad.detach().clone().cpu() for k, p in tr.model.named_parameters()})

        losses = eng.step(torch.tensor(x, dtype=torch.float32, device="cuda"), torch.tensor(label, device="cuda"),
                          before_update=grab).clone().cpu()
        torch.cuda.synchronize()
        merged = L.cv_debug_aux_count(1)
    finally:
        engine.LATENT_AUX = prev_e
        engine.LATENT_CHAIN = prev_c
        L.cv_debug_aux(prev_l)
    return dict(losses=losses, merged=merged, **held), (x, label, ec, es, hp, sd)


def _rel(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("chain,aux_out", [(True, False), (False, False), (False, True)],
                         ids=["chain", "combine-launch", "grad-in-output-loss"])
@pytest.mark.parametrize("aux_lib", [True, False], ids=["merged", "standalone-at-flush"])
def test_aux_schedule_matches_latent_step(aux_lib, chain, aux_out):
    from oracle import cpu_ref as R
    from cvhip import engine
    from test_gpu_declinear import _chain_torch

    prev = engine.LATENT_AUX_OUT
    engine.LATENT_AUX_OUT = aux_out
    try:
        new, inp = _run(True, aux_lib, chain)
    finally:
        engine.LATENT_AUX_OUT = prev
    old, _ = _run(False, True)
    assert new["merged"] == (2 if aux_lib else 0), new["merged"]
    assert old["merged"] == 0
    if chain:  # (d(heads) in memory holds the KL + contrastive terms; the heads backward adds the chain term)
        new["dheads"] = _chain_torch(new["dheads"], new["heads"], new["z"], new["dz"], 16 // 2)
    for k in ("heads", "dheads"):
        assert _rel(new[k], old[k]) < 1e-6, (k, _rel(new[k], old[k]))
    assert _rel(new["losses"][:5], old["losses"][:5]) < 1e-6, (new["losses"][:5], old["losses"][:5])
    worst = max(_rel(new["grads"][k], old["grads"][k]) for k in old["grads"] if float(old["grads"][k].norm()) > 0)
    assert worst < 1e-5, worst
    x, label, ec, es, hp, sd = inp
    o = R.clear_step(R.to_torch(sd), torch.tensor(x), torch.tensor(label), torch.tensor(ec), torch.tensor(es), "VAE",
                     hp)
    for i, k in enumerate(("rec", "kl_c", "kl_s", "c_loss", "s_loss")):
        ref = float(o[k])
        assert abs(float(new["losses"][i]) - ref) <= 1e-4 * max(abs(ref), 1e-3), (k, float(new["losses"][i]), ref)
