"""Per-workgroup timeline of one step-program call INSIDE a step (stamps build): every call of the step
before the target runs eagerly on the step stream, the stamp buffer is cleared, then the target call runs.
Compared with scratch/stamps.py (isolated repeats) this shows what the preceding kernels leave behind.
usage: CVHIP_LIB=scratch/libclearvae_stamps.so python scratch/stamps_instep.py CONFIG CALL..."""
import ctypes, json, sys, os
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
flat = []
for pname, P in bench._programs(G):
    for i, c in enumerate(P.calls):
        flat.append((f"{pname}[{i}]", c))
pos = {lab: k for k, (lab, _) in enumerate(flat)}
s_ = _lib.stream_handle()
q = lambda v: [round(float(v.quantile(x)), 2) for x in (0.0, 0.5, 0.9, 1.0)]
for call in sys.argv[2:]:
    for mode in ("instep", "repeat"):
        out = []
        for rep in range(3):
            if mode == "instep":
                for lab, (name, fn, cargs, _) in flat[:pos[call]]:
                    _lib.check(fn(*cargs, s_), name)
            buf.zero_()
            name, fn, cargs, _ = flat[pos[call]][1]
            _lib.check(fn(*cargs, s_), name)
            torch.cuda.synchronize()
            st = buf.view(-1, 8).cpu()
            used = st[:, 0] > 0
            st = st[used].double()
            t0 = st[:, 0].min()
            ent = (st[:, 0] - t0) * 0.01; pro = (st[:, 1] - st[:, 0]) * 0.01; loop = (st[:, 2] - st[:, 1]) * 0.01
            epi = (st[:, 3] - st[:, 2]) * 0.01; end = (st[:, 3] - t0) * 0.01
            out.append({"wgs": int(used.sum()), "span_us": round(float(end.max()), 2), "entry_q": q(ent),
                        "prologue_q": q(pro), "loop_q": q(loop), "epilogue_q": q(epi), "per_wg_q": q(end - ent),
                        "last_exit_minus_2nd": round(float(end.sort().values[-1] - end.sort().values[-2]), 2)})
        print(json.dumps({"call": call, "mode": mode, "name": name, "runs": out[1:]}))
