import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "clear-vae_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import test_gpu_fallback_paths as T
for off in ([], T.KNOBS):
    for zt in (12, 20, 24):
        try:
            T._run(64, zt, off)
            print(zt, off, "ok", flush=True)
        except AssertionError as e:
            print(zt, off, "FAIL", str(e)[:200], flush=True)
