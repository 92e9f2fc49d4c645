"""The queued NT-Xent phase (cv_ntxent_aux, csrc/cv_aux.hip) is keyed by the stream it was queued for, and the engine
drops it when a program raises before its flush (reference terms: trainer.py:474-479 via losses.py:98-137).

  * queued on stream A, a served direct conv launched on stream B does not take it (cv_debug_aux_count stays 0, the
    phase stays pending); the flush, issued from B, launches it on A; the phase's outputs (row log-sum-exps and the
    contrastive losses of the step) equal those of the normal same-stream schedule bit for bit;
  * a Program that raises between cv_ntxent_aux and its flush leaves nothing queued (cv_ntxent_aux_pending = 0), so
    a later step cannot issue a request that holds the failed step's pointers."""

import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

N = 512


def _engine():
    from oracle import cpu_ref as R
    from cvhip import rng
    from cvhip.engine import ClearStep
    from test_gpu_parity import _fused_trainer

    sd = R.det_state("VAE", 16, 1)
    x, label, ec, es, _ = R.det_inputs(N, 1, 28, 16, 10)
    hp = {"temperature": 0.1, "alpha": 100.0, "beta": 0.125, "ps": True, "loc": 0, "scale": 1}
    tr = _fused_trainer("VAE", 16, 1, sd, hp)
    eng = ClearStep.build(tr, "clear")
    rng.clear_injections()
    X = torch.tensor(x, dtype=torch.float32, device="cuda")
    L = torch.tensor(label, device="cuda")
    eng.graphs_enabled = False
    eng.step(X, L)  # (eager: builds the programs and buffers)
    torch.cuda.synchronize()
    return eng, X, L


def _call(P, i, stream):
    name, fn, args, _ = P.calls[i]
    from cvhip import _lib

    rc = fn(*args, stream)
    if rc != 0:
        _lib.check(rc, name)


def test_phase_stays_on_its_stream():
    from cvhip import _lib

    lib = _lib.lib()
    if not lib.cv_debug_aux(-1):
        pytest.skip("merge disabled in the library (CV_AUX=0)")
    eng, X, L = _engine()
    G = eng.graphs[N]
    ws = G["ws"]
    fwd = G["fwd"]
    names = [c[0] for c in fwd.calls]
    assert "cv_ntxent_aux" in names, names
    q = names.index("cv_ntxent_aux")
    conv = q + 1
    while names[conv].startswith("cv_ntxent_aux"):
        conv += 1
    main = torch.cuda.current_stream()

    # the reference: the program as the engine runs it (queue and served conv on one stream)
    lib.cv_debug_aux_count(1)
    fwd.run(main.cuda_stream)
    torch.cuda.synchronize()
    assert lib.cv_debug_aux_count(1) >= 1
    want_lse = ws.lse[0].clone()
    want_loss = ws.losses[3].clone()

    # again: the phase queued for a side stream, the conv on the main stream
    side = torch.cuda.Stream()
    ws.lse[0].zero_()
    torch.cuda.synchronize()
    for i in range(q):
        _call(fwd, i, main.cuda_stream)
    torch.cuda.synchronize()
    _call(fwd, q, side.cuda_stream)
    assert lib.cv_ntxent_aux_pending() == 1  # (phase 0 queued)
    _call(fwd, conv, main.cuda_stream)
    assert lib.cv_debug_aux_count(1) == 0, "a launch on another stream took the queued phase"
    assert lib.cv_ntxent_aux_pending() == 1
    assert lib.cv_ntxent_aux_flush(ctypes.c_void_p(main.cuda_stream)) == 0
    assert lib.cv_ntxent_aux_pending() == 0
    side.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(ws.lse[0], want_lse)
    # (finish the program so the step's state is whole again; the later phase then queues on the main stream)
    for i in range(conv + 1, len(fwd.calls)):
        if fwd.calls[i][0] != "cv_ntxent_aux_flush" or lib.cv_ntxent_aux_pending():
            _call(fwd, i, main.cuda_stream)
    torch.cuda.synchronize()
    assert lib.cv_ntxent_aux_pending() == 0
    assert torch.isfinite(want_loss).all()


def test_raising_program_drops_the_queued_phase():
    from cvhip import _lib
    from cvhip.plan import Program

    lib = _lib.lib()
    eng, X, L = _engine()
    fwd = eng.graphs[N]["fwd"]
    names = [c[0] for c in fwd.calls]
    q = names.index("cv_ntxent_aux")
    P = Program()
    P.calls = list(fwd.calls[:q + 1])

    def boom(*a):
        raise RuntimeError("injected failure after the queue")

    P.calls.append(("boom", boom, [], 0))
    with pytest.raises(RuntimeError, match="injected"):
        P.run()
    assert lib.cv_ntxent_aux_pending() == 0
    torch.cuda.synchronize()
    # and the engine still steps normally afterwards
    out = eng.step(X, L)
    torch.cuda.synchronize()
    assert torch.isfinite(out[:5]).all()
