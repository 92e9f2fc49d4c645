"""Micro-timing of the latent kernels at MNIST shape (n=512, d=8): rows / grad / combine / fused latent step."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "clear-vae_amd"))
import torch
from cvhip import _lib
from cvhip._lib import cv_ntxent_branch
n, d = int(sys.argv[1]) if len(sys.argv) > 1 else 512, 8
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
heads = torch.randn(n, 4 * d, device=dev, generator=g)
z = torch.randn(n, 2 * d, device=dev, generator=g)
dz = torch.randn(n, 2 * d, device=dev, generator=g) * 1e-3
dheads = torch.zeros(n, 4 * d, device=dev)
losses = torch.zeros(8, device=dev)
lse = torch.zeros(2, 2 * n, device=dev)
lab = torch.randint(0, 10, (n,), device=dev, generator=g)
anneal = torch.zeros(1, dtype=torch.int64, device=dev)
rec = torch.zeros(32, dtype=torch.float64, device=dev)
hb, dh = heads.data_ptr(), dheads.data_ptr()
br = [cv_ntxent_branch(hb, hb + 4 * d, 4 * d, 0, dh, dh + 4 * d, 4 * d, None, 100.0, losses.data_ptr() + 12, lse[0].data_ptr()),
      cv_ntxent_branch(hb + 8 * d, hb + 12 * d, 4 * d, 1, dh + 8 * d, dh + 12 * d, 4 * d, None, 100.0, losses.data_ptr() + 16, lse[1].data_ptr())]
arr = (cv_ntxent_branch * 2)(*br)
s = _lib.stream_handle()
L = _lib.lib()
calls = {
    "rows(2 br)": lambda: _lib.check(L.cv_ntxent(arr, 2, lab.data_ptr(), n, d, 0, ctypes.c_float(0.1), 0, 1, s), "ntx"),
    "grad(2 br)": lambda: _lib.check(L.cv_ntxent(arr, 2, lab.data_ptr(), n, d, 0, ctypes.c_float(0.1), 1, 1, s), "ntx"),
    "rows(1 br)": lambda: _lib.check(L.cv_ntxent(arr, 1, lab.data_ptr(), n, d, 0, ctypes.c_float(0.1), 0, 1, s), "ntx"),
    "combine": lambda: _lib.check(L.cv_latent_combine(heads.data_ptr(), z.data_ptr(), dz.data_ptr(), n, d, ctypes.c_float(0.125), ctypes.c_float(0), ctypes.c_float(1), anneal.data_ptr(), rec.data_ptr(), dheads.data_ptr(), losses.data_ptr(), s), "cmb"),
    "latent_step": lambda: _lib.check(L.cv_latent_step(heads.data_ptr(), z.data_ptr(), dz.data_ptr(), n, d, ctypes.c_float(0.125), ctypes.c_float(0), ctypes.c_float(1), anneal.data_ptr(), rec.data_ptr(), dheads.data_ptr(), losses.data_ptr(), arr, 2, lab.data_ptr(), 0, ctypes.c_float(0.1), s), "lat"),
}
for name, fn in calls.items():
    for _ in range(5): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100): fn()
    e1.record(); torch.cuda.synchronize()
    print(f"{name:14s} {e0.elapsed_time(e1) * 10:.2f} us")
