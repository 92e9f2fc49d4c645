"""Print the step program's call labels with their conv geometry (to pick calls for --only-call)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench, torch
cfgname = sys.argv[1] if len(sys.argv) > 1 else "mnist"
cfg = bench.CONFIGS[cfgname]
res = bench.run_workload(cfgname, cfg, 0, 1, torch.device("cuda", 0), 1, 0, detail=False)
G = res["eng"].graphs[cfg[4]]
for pname, P in bench._programs(G):
    for i, c in enumerate(P.calls):
        extra = ""
        if c[0].startswith("cv_conv"):
            g = c[2][0]._obj
            extra = f"n={g.n} {g.c_in}x{g.h_in} -> {g.c_out}x{g.h_out} T={g.transposed}"
        print(f"{cfgname} {pname}[{i}]:{c[0]} {extra}")
