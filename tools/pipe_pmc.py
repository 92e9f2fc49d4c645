"""50 launches of the device input pipeline at configs[4]'s global batch (1024 x 96x96x3 -> 64x64), for rocprofv3 PMC."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "clear-vae_amd"))
import numpy as np
import torch
from cvhip.data import load_batch
g = np.random.default_rng(0)
imgs = torch.tensor(g.integers(0, 256, size=(4096, 96, 96, 3), dtype=np.uint8), device="cuda")
idx = torch.tensor(g.integers(0, 4096, size=1024), device="cuda")
dst = torch.empty(1024, 3, 64, 64, dtype=torch.float32, device="cuda")
for _ in range(55):
    load_batch(imgs, idx, (64, 64), out=dst)
torch.cuda.synchronize()
print("ok")
