"""Per-workgroup timeline of one step-program call (stamps build): entry, prologue done, main loop done,
exit (s_memrealtime, 100 MHz).  usage: CVHIP_LIB=scratch/libclearvae_stamps.so python scratch/stamps.py CONFIG CALL..."""
import ctypes, json, sys, os
sys.argv += []
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "clear-vae_amd")); sys.path.insert(0, ROOT)
import torch
import bench
from cvhip import _lib

cfgname = sys.argv[1]
cfg = bench.CONFIGS[cfgname]
dev = torch.device("cuda", 0)
res = bench.run_workload(cfgname, cfg, 0, 3, dev, 1, 0, detail=False)
G = res["eng"].graphs[cfg[4]]
L = _lib.lib()
buf = torch.zeros(8 * 65536, dtype=torch.int64, device=dev)
for nm in ("cv_debug_set_stamps", "cv_debug_set_stamps_gather", "cv_debug_set_stamps_scatter",
           "cv_debug_set_stamps_wgrad", "cv_debug_set_stamps_dense"):
    f = getattr(L, nm); f.argtypes = [ctypes.c_void_p]; f.restype = ctypes.c_int
    assert f(buf.data_ptr()) == 0
progs = dict(bench._programs(G))
for call in sys.argv[2:]:
    pname, idx = call.split("[")
    name, fn, cargs, _ = progs[pname].calls[int(idx.rstrip("]"))]
    s_ = _lib.stream_handle()
    for rep in range(3):
        buf.zero_()
        torch.cuda.synchronize()
        _lib.check(fn(*cargs, s_), name)
        torch.cuda.synchronize()
    st = buf.view(-1, 8).cpu()
    used = st[:, 0] > 0
    st = st[used].double()
    t0 = st[:, 0].min()
    ent = (st[:, 0] - t0) * 0.01; pro = (st[:, 1] - st[:, 0]) * 0.01; loop = (st[:, 2] - st[:, 1]) * 0.01
    epi = (st[:, 3] - st[:, 2]) * 0.01; end = (st[:, 3] - t0) * 0.01
    q = lambda v: [round(float(v.quantile(x)), 2) for x in (0.0, 0.5, 0.9, 1.0)]
    print(json.dumps({"call": call, "name": name, "wgs": int(used.sum()), "span_us": round(float(end.max()), 2),
                      "entry_q": q(ent), "prologue_q": q(pro), "loop_q": q(loop), "epilogue_q": q(epi),
                      "per_wg_q": q(end - ent)}))
