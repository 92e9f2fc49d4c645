"""Micro-timing of the fused latent-side kernels (cv_declinear.hip) at the MNIST / VAE64 shapes:
Philox-drawing vs injected eps, and the backward / heads kernels (HIP events, 200 launches)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "clear-vae_amd"))
from cvhip import _lib  # noqa: E402

dev = torch.device("cuda")
s = _lib.stream_handle()


def timeit(fn, reps=200):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for n, d, ch, pix in ((512, 8, 128, 16), (256, 32, 512, 4)):
    F, K, J = ch * pix, 2 * d, 4 * d
    heads = torch.randn(n, 4 * d, device=dev) * 0.3
    W = torch.randn(F, K, device=dev) * 0.1
    b = torch.randn(F, device=dev) * 0.1
    gam, bet = torch.ones(F, device=dev), torch.zeros(F, device=dev)
    rm, rv = torch.zeros(F, device=dev), torch.ones(F, device=dev)
    R = _lib.stat_repl(F)
    stat = torch.zeros(R, 2, F, dtype=torch.float64, device=dev)
    gstat = torch.zeros(R, 2, F, dtype=torch.float64, device=dev)
    bn = _lib.cv_bn(gam.data_ptr(), bet.data_ptr(), stat.data_ptr(), gstat.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                    F, n, 1, 1e-5, None, None, None)
    lin = _lib.cv_linear(n, K, F, 1, 0, pix, ch, 0)
    off = torch.zeros(2, dtype=torch.int64, device=dev)
    eps = torch.randn(n, K, device=dev)
    z = torch.empty(n, K, device=dev)
    h = torch.empty(n, F, device=dev)
    ah = torch.empty(n, F, device=dev)
    L = _lib.lib()

    def fwd(e):
        return lambda: L.cv_decoder_input_forward(ctypes.byref(lin), heads.data_ptr(), e, ctypes.c_uint64(1),
                                                  off.data_ptr(), z.data_ptr(), W.data_ptr(), b.data_ptr(),
                                                  ctypes.byref(bn), stat.data_ptr(), h.data_ptr(), ah.data_ptr(), s)

    def fwd_z():
        return L.cv_decoder_input_forward(ctypes.byref(lin), None, None, ctypes.c_uint64(1), None, z.data_ptr(),
                                          W.data_ptr(), b.data_ptr(), ctypes.byref(bn), stat.data_ptr(),
                                          h.data_ptr(), ah.data_ptr(), s)

    ga = torch.randn(n, F, device=dev)
    gw = torch.zeros(F, K, device=dev)

    def bwd():
        return L.cv_decoder_input_backward(ctypes.byref(lin), ga.data_ptr(), h.data_ptr(), ctypes.byref(bn),
                                           gstat.data_ptr(), z.data_ptr(), gw.data_ptr(), W.data_ptr(), None, s)

    def rep():
        return L.cv_reparam_forward(heads.data_ptr(), n, d, None, ctypes.c_uint64(1), off.data_ptr(), z.data_ptr(),
                                    None, s)
    C = ch
    Fh = F
    dheads = torch.randn(n, J, device=dev)
    Wh = torch.randn(J, Fh, device=dev) * 0.05
    y = torch.randn(n, Fh, device=dev)
    gC, bC = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    stc = torch.zeros(_lib.stat_repl(C), 2, C, dtype=torch.float64, device=dev)
    stc[0, 1] = n * pix
    gsc = torch.zeros_like(stc)
    bnc = _lib.cv_bn(gC.data_ptr(), bC.data_ptr(), stc.data_ptr(), gsc.data_ptr(), rm.data_ptr(), rv.data_ptr(), C,
                     n * pix, 1, 1e-5, None, None, None)
    linh = _lib.cv_linear(n, Fh, J, pix, C, 1, 0, 0)
    gin = torch.empty(n, Fh, device=dev)
    gwh = torch.zeros(J, Fh, device=dev)
    gbh = torch.zeros(J, device=dev)

    def hb():
        return L.cv_heads_backward(ctypes.byref(linh), dheads.data_ptr(), Wh.data_ptr(), y.data_ptr(),
                                   ctypes.byref(bnc), gin.data_ptr(), gsc.data_ptr(), gwh.data_ptr(), gbh.data_ptr(), s)

    print(f"n={n} d={d}: fwd philox {timeit(fwd(None)):.1f} us, fwd eps-injected {timeit(fwd(eps.data_ptr())):.1f} us, "
          f"fwd z-given {timeit(fwd_z):.1f} us, reparam alone {timeit(rep):.1f} us, bwd {timeit(bwd):.1f} us, "
          f"heads bwd {timeit(hb):.1f} us", flush=True)
