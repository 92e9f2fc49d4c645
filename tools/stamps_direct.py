"""Per-workgroup phase timeline of direct-conv (and edge_scatter: weights+constants, staged, MFMA, stores, stats)
calls INSIDE a step (stamps build, cv_direct.hip CV_STAMPS):
every call of the step before the target runs eagerly on the step stream, the stamp buffer is cleared, then the
target call runs.  Phases: constants (entry -> BN constants staged), region (-> region staged and the ring's first
stages landed), stages (-> last weight stage), epilogue (-> output stores issued), stats (-> exit).
usage: CVHIP_LIB=scratch/libclearvae_stamps.so python tools/stamps_direct.py CONFIG CALL..."""
import ctypes, json, os, sys
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
for nm in ("cv_debug_set_stamps_direct", "cv_debug_set_stamps_edge"):
    f = getattr(L, nm)
    f.argtypes = [ctypes.c_void_p]
    f.restype = ctypes.c_int
    assert f(buf.data_ptr()) == 0
flat = []
for pname, P in bench._programs(G):
    for i, c in enumerate(P.calls):
        flat.append((f"{pname}[{i}]", c))
pos = {lab: k for k, (lab, _) in enumerate(flat)}


def _edge_label():  # "@edge": the forward ConvTranspose2d back to the image (<= 4 channels)
    for lab, c in flat:
        if lab.startswith("fwd") and c[0].startswith("cv_conv"):
            g = c[2][0]._obj
            if g.transposed and g.c_out <= 4:
                return lab
    raise SystemExit("no image-side ConvTranspose2d forward call")


s_ = _lib.stream_handle()
q = lambda v: [round(float(v.quantile(x)), 2) for x in (0.0, 0.5, 0.9, 1.0)]
names = ("constants", "region", "stages", "epilogue", "stats")
for call in sys.argv[2:]:
    if call == "@edge":
        call = _edge_label()
    out = []
    for rep in range(3):
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
        r = {"wgs": int(used.sum()), "span_us": round(float((st[:, 5] - t0).max()) * 0.01, 2),
             "entry_q": q((st[:, 0] - t0) * 0.01), "per_wg_q": q((st[:, 5] - st[:, 0]) * 0.01)}
        for k, nm in enumerate(names):
            r[nm + "_q"] = q((st[:, k + 1] - st[:, k]) * 0.01)
        out.append(r)
    print(json.dumps({"call": call, "name": name, "runs": out[1:]}))
