"""Times the real reference's training step (CLEARVAETrainer._train / ClearMIMVAETrainer._train, imported from
/root/reference in the development container only) next to oracle/ref_loop.RefLoop on the same synthetic
batches and thread count, to calibrate bench.py's cpu_baseline.  Not a test; run by hand:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/calibrate_cpu.py [--threads 8] [--config mnist|celeba-mim]

Prints one JSON line per loop with img/s."""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

CFG = {  # arch, z, C, hw, batch, mode, labels, hp
    "mnist": ("VAE", 16, 1, 28, 512, "clear", 10, dict(beta=1 / 8, vae_lr=5e-4, alpha=100.0, temperature=0.1, ps=True)),
    "celeba-mim": ("VAE64", 64, 3, 64, 256, "mim", 4,
                   dict(beta=1 / 32, vae_lr=3e-5, alpha=100.0, temperature=0.1, la=3.0, mi_lr=2e-3)),
}


def batches(cfg, k):
    arch, z, C, hw, B, mode, nl, hp = cfg
    g = torch.Generator().manual_seed(1000)
    return [(torch.rand(B, C, hw, hw, generator=g), torch.randint(0, nl, (B, 1), generator=g)) for _ in range(k)]


def time_port(cfg, data, warm=2):
    from oracle.ref_loop import RefLoop

    arch, z, C, hw, B, mode, nl, hp = cfg
    loop = RefLoop(arch, z, C, mode, hp)
    for X, y in data[:warm]:
        loop.step(X, y.reshape(-1))
    t0 = time.perf_counter()
    for X, y in data[warm:]:
        loop.step(X, y.reshape(-1))
    return B * (len(data) - warm) / (time.perf_counter() - t0)


def time_reference(cfg, data, warm=2):
    sys.path.insert(0, "/root/reference/code")
    from src.utils.trainer_utils import get_clearmimvae_trainer, get_clearvae_trainer

    arch, z, C, hw, B, mode, nl, hp = cfg
    dev = torch.device("cpu")
    if mode == "clear":
        tr = get_clearvae_trainer(beta=hp["beta"], ps=hp["ps"], vae_lr=hp["vae_lr"], z_dim=z, alpha=hp["alpha"],
                                  temperature=hp["temperature"], device=dev, vae_arch=arch, in_channel=C)
        run = lambda d: tr._train(d, False, 0)  # noqa: E731
    else:
        tr = get_clearmimvae_trainer(beta=hp["beta"], mi_estimator="CLUBSample", la=hp["la"], vae_lr=hp["vae_lr"],
                                     mi_estimator_lr=hp["mi_lr"], z_dim=z, alpha=hp["alpha"],
                                     temperature=hp["temperature"], device=dev, vae_arch=arch, in_channel=C)
        run = lambda d: tr._train(d, False, 0, [], [])  # noqa: E731
    run(data[:warm])
    t0 = time.perf_counter()
    run(data[warm:])
    return B * (len(data) - warm) / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--config", default="mnist", choices=sorted(CFG))
    ap.add_argument("--steps", type=int, default=12)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    cfg = CFG[args.config]
    data = batches(cfg, args.steps + 2)
    port, ref = [], []
    for _ in range(3):  # alternate, keep the best of each (thread-pool / allocator warm-up, host noise)
        ref.append(time_reference(cfg, data))
        port.append(time_port(cfg, data))
    port, ref = max(port), max(ref)
    print(json.dumps({"config": args.config, "threads": args.threads, "reference_img_s": round(ref, 1),
                      "ref_loop_img_s": round(port, 1), "ratio": round(port / ref, 3)}))


if __name__ == "__main__":
    main()
