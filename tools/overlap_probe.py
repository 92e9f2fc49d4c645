"""Can two independent step calls share the GPU?  For pairs of calls of the MNIST step that depend only on
earlier calls (a layer's backward-data and its weight gradient), time REPS repetitions of
  seq: A then B on one stream
  par: A on stream 1 || B on stream 2 (an event edge from stream 1 before each pair, one back after)
  free: A x REPS on stream 1 || B x REPS on stream 2, joined only at the ends (true kernel concurrency)
with HIP events.  usage: python tools/overlap_probe.py CONFIG "A,B" ["A,B" ...]"""
import json, os, sys
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
calls = {}
for pname, P in bench._programs(G):
    for i, c in enumerate(P.calls):
        calls[f"{pname}[{i}]"] = c
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
REPS = 50


def run(c, s):
    name, fn, cargs, _ = c
    _lib.check(fn(*cargs, s.cuda_stream), name)


for pair in sys.argv[2:]:
    a, b = pair.split(",")
    A, B = calls[a], calls[b]
    out = {"pair": pair, "names": [A[0], B[0]]}
    for mode in ("seq", "par", "free", "A", "B", "free"):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s1)
        for _ in range(REPS):
            if mode == "seq":
                run(A, s1); run(B, s1)
            elif mode == "A":
                run(A, s1)
            elif mode == "B":
                run(B, s1)
            elif mode == "free":  # the two streams' queues run unsynchronised between the end points
                if _ == 0:
                    ev = torch.cuda.Event()
                    ev.record(s1)
                    s2.wait_event(ev)
                run(A, s1); run(B, s2)
                if _ == REPS - 1:
                    ev2 = torch.cuda.Event()
                    ev2.record(s2)
                    s1.wait_event(ev2)
            else:
                ev = torch.cuda.Event()
                ev.record(s1)
                s2.wait_event(ev)
                run(A, s1); run(B, s2)
                ev2 = torch.cuda.Event()
                ev2.record(s2)
                s1.wait_event(ev2)
        e1.record(s1)
        torch.cuda.synchronize()
        out[mode] = round(e0.elapsed_time(e1) / REPS * 1e3, 2)
    print(json.dumps(out), flush=True)
