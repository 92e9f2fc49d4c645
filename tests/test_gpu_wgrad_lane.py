"""Deferred weight gradients on side stream 1 (cvhip/engine.py WGRAD_LANE, cv_conv_backward_deferred_kpack_side)
against the one-stream order (WGRAD_LANE = 0).  Reference step: trainer.py:452-484 (CLEAR-VAE), :842-888
(CLEAR-MIM).

Same weights, same injected noise, two fused steps (the first eager, the second a graph replay) on VAE64 (n = 64)
and VAE (n = 128), CLEAR-VAE and CLEAR-MIM:
  * the side-stream form really issues the side calls (the interior layers' pairs; with WGRAD_LANE = 2 the
    decoder's first ConvTranspose2d too);
  * the step losses, the gradient and parameter arenas after each step are bit-identical to the one-stream
    form's: the weight-gradient launches run the same kernels on the same inputs, only on another queue, and
    cv_step_reduce sums their partials after the join in the same order."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(lane, arch, zt, C, hw, n, mode, split=False, adam_pack=True):
    from oracle import cpu_ref as R
    from cvhip import engine, rng
    from cvhip.engine import ClearStep
    from test_gpu_parity import _fused_trainer

    prev = engine.WGRAD_LANE, engine.SPLIT_UPDATE, engine.ADAM_PACK
    engine.WGRAD_LANE, engine.SPLIT_UPDATE, engine.ADAM_PACK = lane, split, adam_pack
    try:
        torch.manual_seed(4321)
        rng.clear_injections()
        rng.reset_counters()
        sd = R.det_state(arch, zt, C)
        x, label, _, _, _ = R.det_inputs(n, C, hw, zt, 4)
        hp = {"temperature": 0.1, "beta": 1 / 32, "loc": 0, "scale": 1, "alpha": 100.0, "lambda": 3.0, "ps": True}
        kw = dict(mode="mim", kind="CLUBSample", lr=3e-5) if mode == "mim" else {}
        tr = _fused_trainer(arch, zt, C, sd, hp, **kw)
        eng = ClearStep.build(tr, mode)
        assert eng is not None
        X = torch.tensor(x, dtype=torch.float32, device="cuda")
        L = torch.tensor(label, device="cuda")
        res = []
        for _ in range(2):
            out = eng.step(X, L)
            torch.cuda.synchronize()
            lo = out[0] if isinstance(out, tuple) else out
            res.append(dict(loss=lo[:6].cpu().double().numpy(), grad=eng.arena.grad.double().cpu().numpy(),
                            flat=eng.arena.flat.double().cpu().numpy(),
                            m=eng.adam.m.double().cpu().numpy(), v=eng.adam.v.double().cpu().numpy(),
                            counters=np.array([float(eng.adam.step.view(-1)[0]), float(eng.anneal.view(-1)[0])]),
                            bufs=np.concatenate([b.double().cpu().reshape(-1).numpy()
                                                 for _, b in tr.model.named_buffers()])))
        G = eng.graphs[n]
        names = [c[0] for P in (G["dec"], G["enc"], G["upd"]) for c in P.calls]
        return dict(res=res, names=names, replayed="graphs" in G)
    finally:
        engine.WGRAD_LANE, engine.SPLIT_UPDATE, engine.ADAM_PACK = prev


@pytest.mark.parametrize("arch,zt,C,hw,n,mode", [("VAE64", 64, 3, 64, 64, "clear"), ("VAE", 16, 1, 28, 128, "clear"),
                                                  ("VAE64", 64, 3, 64, 64, "mim")])
def test_side_stream_weight_gradients_match_one_stream(arch, zt, C, hw, n, mode):
    base = _run(0, arch, zt, C, hw, n, mode)
    assert "cv_conv_backward_deferred_kpack_side" not in base["names"]
    for lane in (1, 2):
        r = _run(lane, arch, zt, C, hw, n, mode)
        k = r["names"].count("cv_conv_backward_deferred_kpack_side")
        assert k >= 1, r["names"]
        assert r["replayed"] and base["replayed"]
        for step, (ra, rb) in enumerate(zip(r["res"], base["res"])):
            for key in ("loss", "grad", "flat"):
                assert np.array_equal(ra[key], rb[key]), (lane, step, key,
                                                          float(np.abs(ra[key] - rb[key]).max()))


@pytest.mark.parametrize("arch,zt,C,hw,n,mode", [("VAE64", 64, 3, 64, 64, "clear"), ("VAE", 16, 1, 28, 128, "clear"),
                                                  ("VAE64", 64, 3, 64, 64, "mim")])
def test_split_update_matches_one_update(arch, zt, C, hw, n, mode):
    """The decoder bucket's reduction and Adam part on side lane 2 (engine SPLIT_UPDATE, cv_adam_pack_step_part):
    losses, gradients, parameters, Adam moments, the step / annealer counters and the BatchNorm buffers
    bit-identical to the one-update step's after each of two steps (the same per-element arithmetic over the same
    elements; the counters advance once, in the encoder part)."""
    base = _run(2, arch, zt, C, hw, n, mode)
    r = _run(2, arch, zt, C, hw, n, mode, split=True)
    assert "cv_adam_pack_step_part" in r["names"] and "cv_adam_pack_step_part" not in base["names"], r["names"]
    for step, (ra, rb) in enumerate(zip(r["res"], base["res"])):
        for key in rb:
            assert np.array_equal(ra[key], rb[key]), (step, key, float(np.abs(ra[key] - rb[key]).max()))


@pytest.mark.parametrize("arch,zt,C,hw,n", [("VAE64", 64, 3, 64, 64), ("VAE", 16, 1, 28, 128)])
def test_separate_adam_matches_fused_adam_pack(arch, zt, C, hw, n):
    """CVHIP_ADAM_PACK=0 (a packing launch at each step start and the plain Adam kernel) against the Adam launch
    that packs (the default): the same step, one optimizer update per step (counters equal), parameters within
    1e-6 relative (the two Adam kernels share the arithmetic; the compiler may contract it differently)."""
    a = _run(1, arch, zt, C, hw, n, "clear", adam_pack=False)
    b = _run(1, arch, zt, C, hw, n, "clear")
    for step, (ra, rb) in enumerate(zip(a["res"], b["res"])):
        assert np.array_equal(ra["counters"], rb["counters"]), (step, ra["counters"], rb["counters"])
        for key in ("loss", "flat", "m", "v"):
            scale = max(float(np.abs(rb[key]).max()), 1e-30)
            assert float(np.abs(ra[key] - rb[key]).max()) <= 1e-6 * scale, (step, key)
