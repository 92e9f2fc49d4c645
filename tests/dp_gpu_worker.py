"""Worker of tests/test_gpu_dp.py: one rank of a world-2 data-parallel fused step on the single GPU.

Both ranks share cuda:0 and talk over gloo (which accepts device tensors and stages them through the
host), so the engine's own DP code runs end to end: the construction-time broadcast of rank 0's arena,
the segmented step with the decoder bucket all-reduced while the encoder backward runs, the 1/world
gradient scale applied inside cv_adam_step and, in CLEAR-MIM, the estimator all-reduce inside each of
the 5 estimator updates (cvhip/engine.py `_segments`, `make_learn_dp`)."""

import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "clear-vae_amd"), ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def _np(t):
    return t.detach().double().cpu().numpy().copy()


def run(rank, world, port, q, mode, n_global, kind, arch="VAE", precision="fp32"):
    try:
        import numpy as np
        import torch
        import torch.distributed as dist

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(2)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from cvhip import dist as cvd
        from cvhip import rng
        from cvhip.engine import ClearStep
        from oracle import cpu_ref as R
        from src.models.mi_estimator import CLUBSample, L1OutUB
        from cvhip.plan import set_precision
        from src.models.vae import VAE, VAE64
        from src.trainer import ClearMIMVAETrainer, ClearTCVAETrainer, CLEARVAETrainer, HierarchicalVAETrainer

        zt, C = (16, 1) if arch == "VAE" else (64, 3)
        hw = R.IMAGE[arch]
        sd = R.det_state(arch, zt, C)
        if rank != 0:  # a different start on rank 1: the engine must adopt rank 0's weights
            sd = {k: (v * 1.25 if np.asarray(v).dtype != np.int64 else v) for k, v in sd.items()}
        vae = (VAE if arch == "VAE" else VAE64)(zt, C, group_mode=kind if mode == "group" else None).cuda()
        set_precision(vae, precision)
        vae.load_state_dict({k: torch.as_tensor(np.asarray(v)).float() if np.asarray(v).dtype != np.int64
                             else torch.as_tensor(np.asarray(v)) for k, v in sd.items()})
        opt = torch.optim.Adam(vae.parameters(), lr=5e-4)
        dev = torch.device("cuda", 0)
        if mode == "clear":
            hp = {"temperature": 0.1, "alpha": 100.0, "beta": 0.125, "ps": True, "loc": 0, "scale": 1}
            tr = CLEARVAETrainer(vae, opt, "cosine", hp, 1, dev)
        elif mode == "group":
            tr = HierarchicalVAETrainer(vae, opt, {"beta": 0.125, "loc": 0, "scale": 1}, 1, dev)
        elif mode == "tc":
            hp = {"temperature": 0.1, "beta": 0.125, "loc": 0, "scale": 1, "alpha": 100.0, "lambda": 3.0}
            disc = torch.nn.Sequential(torch.nn.Linear(zt, zt), torch.nn.ReLU(), torch.nn.Linear(zt, 1),
                                       torch.nn.Sigmoid()).cuda()
            dd = R.det_disc(zt)
            if rank != 0:
                dd = {k: v * 0.5 for k, v in dd.items()}
            disc.load_state_dict({k: torch.tensor(v, dtype=torch.float32) for k, v in dd.items()})
            fopt = torch.optim.Adam(disc.parameters(), lr=1e-3)
            tr = ClearTCVAETrainer(vae, disc, {"vae_optim": opt, "factor_optim": fopt}, "cosine", hp, 1, dev)
        else:
            hp = {"temperature": 0.1, "beta": 0.125, "loc": 0, "scale": 1, "alpha": 100.0, "lambda": 3.0}
            est = (CLUBSample if kind == "CLUBSample" else L1OutUB)(zt // 2, zt // 2, zt).cuda()
            md = R.det_mlp(zt // 2, zt)
            if rank != 0:
                md = {k: v * 0.5 for k, v in md.items()}
            est.load_state_dict({k: torch.tensor(v, dtype=torch.float32) for k, v in md.items()})
            eopt = torch.optim.Adam(est.parameters(), lr=2e-3)
            tr = ClearMIMVAETrainer(vae, est, {"vae_optim": opt, "mi_estimator_optim": eopt}, "cosine", hp, 1, dev)
        eng = ClearStep.build(tr, mode)
        assert eng is not None and eng.world == world, "fused DP engine not built"
        assert eng.spec.mma == (1 if precision == "bf16" else 0)
        assert len(eng.buckets.bounds) == 3  # decoder, deep encoder, shallow encoder
        out = {"p0": {k: _np(v) for k, v in vae.state_dict().items() if "running" not in k and "num_b" not in k}}
        if mode in ("mim", "tc"):
            out["e0"] = _np(eng.est_arena.flat)

        # step 1: injected noise (eager segments), this rank's contiguous shard of the global batch
        x, label, ec, es, perm = R.det_inputs(n_global, C, hw, zt, 4, seed=21)
        lo, hi = cvd.shard_bounds(n_global, rank, world)
        n = hi - lo
        rng.clear_injections()
        if mode == "clear":
            rng.inject_noise([torch.tensor(ec[lo:hi], dtype=torch.float32), torch.tensor(es[lo:hi], dtype=torch.float32)])
        elif mode == "group":  # content noise rows in this shard's group order
            rng.inject_noise([R.group_order_noise(label[lo:hi], torch.tensor(ec[lo:hi])).float(),
                              torch.tensor(es[lo:hi], dtype=torch.float32)])
        elif mode == "tc":
            gen = np.random.default_rng(6)
            a2, b2 = gen.standard_normal((n_global, zt // 2)), gen.standard_normal((n_global, zt // 2))
            rng.inject_noise([torch.tensor(t[lo:hi], dtype=torch.float32) for t in (ec, es, a2, b2)])
        else:
            gen = np.random.default_rng(5)
            noises = [(ec, es)] + [(gen.standard_normal((n_global, zt // 2)), gen.standard_normal((n_global, zt // 2)))
                                   for _ in range(5)]
            rng.inject_noise([torch.tensor(a[lo:hi], dtype=torch.float32) for pair in noises for a in pair])
            lperm = np.random.default_rng(100 + rank).permutation(n).astype(np.int64)
            rng.inject_perm([torch.tensor(lperm)])
            out["perm"] = lperm
        X = torch.tensor(x[lo:hi], dtype=torch.float32, device=dev)
        L = torch.tensor(label[lo:hi], device=dev)
        held = {}

        def read_masks():  # the ReLU activity of this rank's shard, with the pre-Adam BN affine (tests/maskpin.py)
            from maskpin import device_masks

            held["m"] = device_masks(eng, eng.last_workspace(n), n)

        res = eng.step(X, L, before_update=read_masks)
        torch.cuda.synchronize()
        from maskpin import masks_to_numpy

        out["masks"] = masks_to_numpy(held["m"])
        if mode in ("clear", "group"):
            out["losses"] = _np(res)
        else:
            out["losses"], out["learn"] = _np(res[0]), _np(res[1])
            out["e1"] = _np(eng.est_arena.flat)
        # the arena gradient holds the all-reduced SUM (the 1/world scale is applied inside Adam)
        out["grad"] = {k: _np(p.grad) / world for k, p in vae.named_parameters()}
        out["p1"] = {k: _np(p) for k, p in vae.named_parameters()}
        out["bounds"] = (lo, hi)

        # steps 2-3: device noise, graph capture + replay of the DP segments
        for s in range(2):
            x2, l2, _, _, _ = R.det_inputs(n_global, C, hw, zt, 4, seed=30 + s)
            eng.step(torch.tensor(x2[lo:hi], dtype=torch.float32, device=dev), torch.tensor(l2[lo:hi], device=dev))
        torch.cuda.synchronize()
        out["graphs"] = "graphs" in eng.graphs[n]
        if mode in ("clear", "tc"):  # the device noise of the last step, eps = (z - mu) / exp(logvar / 2)
            ws = eng.last_workspace(n)
            d = zt // 2
            h, z = ws.heads.double().cpu(), ws.z.double().cpu()
            out["eps"] = ((z[:, :d] - h[:, :d]) / torch.exp(0.5 * h[:, d:2 * d])).numpy()
        out["p3"] = _np(eng.arena.flat)
        if mode in ("mim", "tc"):
            out["e3"] = _np(eng.est_arena.flat)
        eng.sync_host_state()
        out["opt_step"] = int(float(opt.state[next(vae.parameters())]["step"]))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out, None))
    except Exception:  # pragma: no cover
        q.put((rank, None, traceback.format_exc()))
