import json, sys, os
sys.path.insert(0, os.getcwd())
import bench, torch
for n, hw in ((1024, 96), (128, 96), (128, 227)):
    r = bench.pipeline_pass(torch.device("cuda"), n=n, hw=hw, cpu_budget_s=0.5)
    print(n, hw, r["us_per_batch"], r["roofline"]["achieved"], r["roofline"]["frac"], r["cpu_reference"]["images_per_s"])
