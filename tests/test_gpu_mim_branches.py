"""CLEAR-MIM's estimator updates with their decoder forwards on side lanes of the step graph (cvhip/engine.py
MIM_BRANCHES, make_learn_branched) against the sequential form (MIM_BRANCHES = 0).  Reference: trainer.py:873-888
(five `vae(X)` train-mode forwards, each updating the BatchNorm running statistics, each followed by one estimator
learning step on its own z).

Same weights, same Philox stream (counters reset, same seed), CLUB-S and L1Out on VAE64 and VAE, two steps (the
first eager, the second a graph replay):
  * the branched step really runs its decoder forwards on side lanes (the learn program has side-lane calls);
  * the step losses, the five learning losses, the VAE and estimator parameter arenas are bit-identical to the
    sequential form's after each step (the same kernels on the same inputs, and a fused step without
    order-dependent sums: tests/test_gpu_determinism.py); num_batches_tracked equal; every BatchNorm running mean /
    variance within 1e-6 relative (the five momentum updates in the same order, one launch instead of five: the
    compiler may contract m * mean + (1 - m) * r into an fma differently in the two kernels, an ulp apart)"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(branches, arch, zt, C, hw, n, kind):
    from oracle import cpu_ref as R
    from cvhip import engine, rng
    from cvhip.engine import ClearStep
    from test_gpu_parity import _fused_trainer

    prev = engine.MIM_BRANCHES
    engine.MIM_BRANCHES = branches
    try:
        torch.manual_seed(4321)
        rng.clear_injections()
        rng.reset_counters()
        sd = R.det_state(arch, zt, C)
        x, label, _, _, _ = R.det_inputs(n, C, hw, zt, 4)
        hp = {"temperature": 0.1, "beta": 1 / 32, "loc": 0, "scale": 1, "alpha": 100.0, "lambda": 3.0}
        tr = _fused_trainer(arch, zt, C, sd, hp, mode="mim", kind=kind, lr=3e-5)
        eng = ClearStep.build(tr, "mim")
        assert eng is not None
        X = torch.tensor(x, dtype=torch.float32, device="cuda")
        L = torch.tensor(label, device="cuda")
        res = []
        for _ in range(2):
            lo, learn = eng.step(X, L)
            torch.cuda.synchronize()
            res.append(dict(loss=lo[:6].cpu().double().numpy(), learn=learn.cpu().double().numpy(),
                            bufs={k: b.detach().double().cpu().numpy() for k, b in tr.model.named_buffers()},
                            flat=eng.arena.flat.double().cpu().numpy(),
                            est=eng.est_arena.flat.double().cpu().numpy()))
        G = eng.graphs[n]
        lanes = {c[3] for c in G["learn"].calls}
        return dict(res=res, lanes=lanes, replayed="graphs" in G)
    finally:
        engine.MIM_BRANCHES = prev


def _close(a, b, tol):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-3)) <= tol


@pytest.mark.parametrize("arch,zt,C,hw,n,kind", [("VAE64", 64, 3, 64, 64, "CLUBSample"),
                                                  ("VAE", 16, 1, 28, 128, "L1OutUB")])
def test_branched_estimator_forwards_match_sequential(arch, zt, C, hw, n, kind):
    a = _run(2, arch, zt, C, hw, n, kind)
    b = _run(0, arch, zt, C, hw, n, kind)
    assert any(isinstance(v, int) and v >= 1 for v in a["lanes"]), a["lanes"]
    assert not any(isinstance(v, int) and v >= 1 for v in b["lanes"]), b["lanes"]
    assert a["replayed"] and b["replayed"]
    for step, (ra, rb) in enumerate(zip(a["res"], b["res"])):
        assert np.array_equal(ra["loss"], rb["loss"]), (step, ra["loss"], rb["loss"])
        assert np.array_equal(ra["learn"], rb["learn"]), (step, ra["learn"], rb["learn"])
        for k in rb["bufs"]:
            if k.endswith("num_batches_tracked"):
                assert np.array_equal(ra["bufs"][k], rb["bufs"][k]), (step, k)
            else:
                assert _close(ra["bufs"][k], rb["bufs"][k], 1e-6), (step, k)
        assert np.array_equal(ra["flat"], rb["flat"]), step
        assert np.array_equal(ra["est"], rb["est"]), step
