"""Worker of tests/test_gpu_graph_collectives.py: one process, a world-1 RCCL (`nccl`) process group on cuda:0,
the fused engine's data-parallel programs forced on (CVHIP_FORCE_DP=1) so its gradient buckets really go through
RCCL, with or without the whole step captured as one graph (CVHIP_GRAPH_COLLECTIVES, read at import).

Runs `steps` fused steps (the first eager, the rest replayed) on a fixed batch and prints one JSON line: the
losses of every step, a digest of the final parameter / Adam-state arenas, and how the step graph was built."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "clear-vae_amd"), ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main(mode, steps, port, n=64, timed=0):
    import numpy as np
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    torch.manual_seed(1234)  # (the engine's Philox stream is keyed by torch's seed: both runs draw the same noise)
    # (no caller setup for the captured form: the default group is built with whatever event-cache setting the
    # environment holds — the test sets the cache ON — and the engine captures on its own group)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from cvhip.engine import ClearStep
    from oracle import cpu_ref as R
    from src.models.mi_estimator import CLUBSample
    from src.models.vae import VAE
    from src.trainer import ClearMIMVAETrainer, CLEARVAETrainer

    zt, C = 16, 1
    sd = R.det_state("VAE", zt, C)
    vae = VAE(zt, C).cuda()
    vae.load_state_dict({k: torch.as_tensor(np.asarray(v)).float() if np.asarray(v).dtype != np.int64
                         else torch.as_tensor(np.asarray(v)) for k, v in sd.items()})
    opt = torch.optim.Adam(vae.parameters(), lr=5e-4)
    dev = torch.device("cuda", 0)
    if mode == "clear":
        hp = {"temperature": 0.1, "alpha": 100.0, "beta": 0.125, "ps": True, "loc": 0, "scale": 1}
        tr = CLEARVAETrainer(vae, opt, "cosine", hp, 1, dev)
    else:
        hp = {"temperature": 0.1, "beta": 0.125, "loc": 0, "scale": 1, "alpha": 100.0, "lambda": 3.0}
        est = CLUBSample(zt // 2, zt // 2, zt).cuda()
        est.load_state_dict({k: torch.tensor(v, dtype=torch.float32) for k, v in R.det_mlp(zt // 2, zt).items()})
        eopt = torch.optim.Adam(est.parameters(), lr=2e-3)
        tr = ClearMIMVAETrainer(vae, est, {"vae_optim": opt, "mi_estimator_optim": eopt}, "cosine", hp, 1, dev)
    eng = ClearStep.build(tr, mode)
    assert eng is not None and eng.dp and eng.world == 1
    x, label, _, _, _ = R.det_inputs(n, C, 28, zt, 10)
    X = torch.tensor(x, dtype=torch.float32, device=dev)
    L = torch.tensor(label, device=dev)
    losses = []
    for _ in range(steps):
        out = eng.step(X, L)
        lo = out[0] if isinstance(out, tuple) else out
        losses.append([float(v) for v in lo[:6].cpu()])
        if isinstance(out, tuple):
            losses[-1] += [float(v) for v in out[1].cpu()]
    torch.cuda.synchronize()
    ms = None
    if timed:  # (timing only: ms per replayed step)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(timed):
            eng.step(X, L)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / timed
    G = eng.graphs[n]
    digest = {"params": eng.arena.flat.double().sum().item(), "params_abs": eng.arena.flat.double().abs().sum().item(),
              "m": eng.adam.m.double().abs().sum().item(), "v": eng.adam.v.double().abs().sum().item()}
    if mode == "mim":
        digest["est"] = eng.est_arena.flat.double().abs().sum().item()
    flat = eng.arena.flat.cpu().numpy()
    print(json.dumps({"mode": mode, "n": n, "ms_per_step": ms, "losses": losses, "digest": digest, "one_graph": bool(G.get("one_graph")),
                      "ngraphs": len(G.get("graphs", [])), "capture": eng.capture_collectives,
                      "own_group": eng.buckets.group is not None,
                      "flat_head": [float(v) for v in flat[:8]], "flat_hash": float(np.abs(flat).astype(np.float64).sum())}),
          flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), *(int(v) for v in sys.argv[4:6]))
