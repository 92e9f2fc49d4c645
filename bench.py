"""CLEAR-VAE training throughput on MI355X (BASELINE.json metric: "training images/sec at bs=512;
ELBO rel-err vs CPU ref").

Default workload (configs[1]): Styled-MNIST-shaped synthetic batches [512, 1, 28, 28] ~ U[0,1), 10
labels, CLEAR-VAE (VAE, z=16, beta=1/8, lr 5e-4, alpha=100, tau=0.1, ps=True,
code/run_styledmnist_downstream_expr.py:231-238), fp32, one fused HIP training step per batch
(forward, ELBO, 2 contrastive terms, backward, Adam) through CLEARVAETrainer's engine.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config mnist|celeba-mim|celeba]

For N > 1 launch with torch.distributed.run (one process per GPU, RCCL): per-GPU batch fixed
(weak scaling); value = images processed by all ranks / max-over-ranks wall time.
After the timed region: (1) a per-kernel HIP-event pass over the same step program to price the
dominant kernel against its roofline, (2) on rank 0 the CPU baseline (oracle/cpu_ref.py, the
reference's math on torch-CPU) on a bounded sample, plus the ELBO relative error of one HIP step
against the fp64 CPU reference on the same batch / weights / noise.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "clear-vae_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_FP32_TFLOPS = 157.3  # MI355X dense FP32 (MFMA f32 = VALU rate), MI355X_MICROARCH.md
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense BF16 MFMA (no sparsity), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0

CONFIGS = {
    # name: (arch, z, in_ch, hw, batch, mode, labels, hyper, estimator)
    "mnist": ("VAE", 16, 1, 28, 512, "clear", 10,
              dict(beta=1 / 8, vae_lr=5e-4, alpha=100.0, temperature=0.1, ps=True), None),
    "celeba-mim": ("VAE64", 64, 3, 64, 256, "mim", 4,
                   dict(beta=1 / 32, vae_lr=3e-5, alpha=100.0, temperature=0.1, la=3.0, mi_lr=2e-3), "CLUBSample"),
    "celeba": ("VAE64", 64, 3, 64, 256, "clear", 4,
               dict(beta=1 / 32, vae_lr=3e-5, alpha=100.0, temperature=0.1, ps=True), None),
    # configs[4]: Camelyon17 patches resized to 64x64 before the model, bs=1024 over 8 GPUs =
    # 128 per GPU, bf16 contractions
    "camelyon-bf16": ("VAE64", 64, 3, 64, 128, "clear", 2,
                      dict(beta=1 / 32, vae_lr=3e-5, alpha=100.0, temperature=0.1, ps=True, precision="bf16"), None),
}


def make_trainer(cfg, device):
    from src.utils.trainer_utils import get_clearmimvae_trainer, get_clearvae_trainer

    arch, z, C, hw, B, mode, nl, hp, est = cfg
    if mode == "clear":
        return get_clearvae_trainer(beta=hp["beta"], ps=hp["ps"], vae_lr=hp["vae_lr"], z_dim=z, alpha=hp["alpha"],
                                    temperature=hp["temperature"], device=device, vae_arch=arch, in_channel=C,
                                    verbose_period=10**9, precision=hp.get("precision", "fp32"))
    return get_clearmimvae_trainer(beta=hp["beta"], mi_estimator=est, la=hp["la"], vae_lr=hp["vae_lr"],
                                   mi_estimator_lr=hp["mi_lr"], z_dim=z, alpha=hp["alpha"],
                                   temperature=hp["temperature"], device=device, vae_arch=arch, in_channel=C,
                                   verbose_period=10**9, precision=hp.get("precision", "fp32"))


def conv_flops_per_image(spec):
    """Algorithmic FLOPs of one training step per image (MAC x 2; fwd + bwd-data + bwd-weight)."""
    f = 0
    for c in spec.enc + spec.dec:
        k = c.mod.kernel_size[0] * c.mod.kernel_size[1]
        if c.transposed:
            macs = c.h_in * c.w_in * c.c_in * c.c_out * k
        else:
            macs = c.h_out * c.w_out * c.c_out * c.c_in * k
        f += 2 * macs
    f += 2 * spec.F * 4 * spec.d + 2 * 2 * spec.d * spec.dec_lin.out_features
    return 3 * f


def kernel_pass(engine, G, reps=20, rounds=3):
    """Per-call device time of the step program: each C-ABI call is captured REPS times back to back
    into its own HIP graph (torch.cuda.CUDAGraph on the stream the kernels are launched on) and the
    graph replay is bracketed by HIP events, so the average excludes host launch gaps.  Returns
    {call label: mean ms per launch}.  (Repeating a call perturbs the workspace; run after timing.)"""
    from cvhip import _lib

    progs = [("fwd", G["fwd"]), ("dec", G["dec"]), ("lat", G["lat"]), ("enc", G["enc"]), ("upd", G["upd"])]
    learn = G.get("learn")
    if isinstance(learn, list):  # data-parallel CLEAR-MIM: (gradient, Adam) program pairs
        for j, (gp, ap) in enumerate(learn):
            progs += [(f"learn{j}g", gp), (f"learn{j}a", ap)]
    elif learn is not None:
        progs.append(("learn", learn))
    times = {}
    for pname, P in progs:
        for i, (name, fn, args, _lane) in enumerate(P.calls):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                s = _lib.stream_handle()
                for _ in range(reps):
                    _lib.check(fn(*args, s), name)
            g.replay()
            torch.cuda.synchronize()
            best = None
            for _ in range(rounds):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                best = ms if best is None else min(best, ms)
            times[f"{pname}[{i}]:{name}"] = best
            del g
    return times


def gemm_flops_of(label, G, engine):
    """Algorithmic FLOPs of one igemm call from its program position (conv / linear layers)."""
    pname, rest = label.split("[", 1)
    idx = int(rest.split("]")[0])
    if not hasattr(G.get(pname), "calls"):
        return None
    name, fn, args, _lane = G[pname].calls[idx]
    if name.startswith("cv_conv_"):
        g = args[0]._obj
        k = g.kh * g.kw
        if g.transposed:
            macs = g.n * g.h_in * g.w_in * g.c_in * g.c_out * k
        else:
            macs = g.n * g.h_out * g.w_out * g.c_out * g.c_in * k
        return 2.0 * macs
    if name.startswith("cv_linear_"):
        g = args[0]._obj
        return 2.0 * g.n * g.in_features * g.out_features
    return None


def cpu_baseline(cfg, steps_budget_s=15.0):
    """Reference math on the host (oracle/cpu_ref.py, torch-CPU fp32) on a bounded sample."""
    import numpy as np

    from oracle import cpu_ref as R

    arch, z, C, hw, B, mode, nl, hp, est = cfg
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
    sd = R.det_state(arch, z, C)
    P = R.to_torch(sd, torch.float32)
    params = [v for v in P.values() if isinstance(v, torch.Tensor) and v.requires_grad]
    opt = torch.optim.Adam(params, lr=hp["vae_lr"])
    hpp = dict(temperature=hp["temperature"], alpha=hp["alpha"], beta=hp["beta"], ps=hp.get("ps", True),
               **({"lambda": hp["la"]} if mode == "mim" else {}))
    M = R.to_torch(R.det_mlp(z // 2, z), torch.float32) if mode == "mim" else None
    steps = 0
    work = 0.0
    t0 = time.perf_counter()
    while True:
        x, label, ec, es, perm = R.det_inputs(B, C, hw, z, nl, seed=1000 + steps)
        xt, lt = torch.tensor(x, dtype=torch.float32), torch.tensor(label)
        ect, est_ = torch.tensor(ec, dtype=torch.float32), torch.tensor(es, dtype=torch.float32)
        t_s = time.perf_counter()
        if mode == "clear":
            o = R.clear_step(P, xt, lt, ect, est_, arch, hpp, step=steps)
        else:
            o = R.mim_step(P, M, xt, lt, ect, est_, torch.tensor(perm), arch, hpp, step=steps)
        for p, g in zip(params, o["grads"].values()):
            p.grad = g
        opt.step()
        if mode == "mim":  # the 5 estimator updates each need a VAE forward (trainer.py:874-888)
            with torch.no_grad():
                for _ in range(5):
                    R.vae_forward(P, xt, ect, est_, arch, True)
        steps += 1
        work += time.perf_counter() - t_s
        if time.perf_counter() - t0 > steps_budget_s or steps >= 200:
            break
    return {"value": round(B * steps / work, 1), "unit": "images/s", "cores": torch.get_num_threads(),
            "kind": "port", "sample": f"{steps} steps x bs={B} {arch} {mode} fp32 (oracle/cpu_ref.py + torch Adam)"}


def elbo_rel_err(cfg, device):
    """One fused HIP step on a fixed batch with injected noise vs the fp64 CPU reference."""
    import numpy as np

    from cvhip import rng
    from cvhip.engine import ClearStep
    from oracle import cpu_ref as R

    arch, z, C, hw, B, mode, nl, hp, est = cfg
    if mode != "clear":
        return None
    tr = make_trainer(cfg, device)
    sd = R.det_state(arch, z, C)
    tr.model.load_state_dict({k: torch.as_tensor(np.asarray(v)).float() if np.asarray(v).dtype != np.int64
                              else torch.as_tensor(np.asarray(v)) for k, v in sd.items()})
    eng = ClearStep.build(tr, "clear")
    x, label, ec, es, perm = R.det_inputs(B, C, hw, z, nl, seed=77)
    rng.clear_injections()
    rng.inject_noise([torch.tensor(ec, dtype=torch.float32), torch.tensor(es, dtype=torch.float32)])
    L = eng.step(torch.tensor(x, dtype=torch.float32, device=device), torch.tensor(label, device=device)).cpu()
    hpp = dict(temperature=hp["temperature"], alpha=hp["alpha"], beta=hp["beta"], ps=hp["ps"])
    o = R.clear_step(R.to_torch(sd), torch.tensor(x), torch.tensor(label), torch.tensor(ec), torch.tensor(es), arch,
                     hpp)
    w = R.anneal_weight(0, hp["beta"])
    elbo_hip = float(L[0]) + w * float(L[1]) + w * float(L[2])
    elbo_ref = float(o["rec"]) + w * float(o["kl_c"]) + w * float(o["kl_s"])
    return abs(elbo_hip - elbo_ref) / abs(elbo_ref)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="mnist", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-pass", action="store_true")
    ap.add_argument("--kernel-table", default=None, help="write the per-call timing table to this file")
    ap.add_argument("--only-call", default=None,
                    help="profiling mode: after warmup, launch this step-program call (e.g. 'enc[4]') --reps "
                         "times back to back and exit (for rocprofv3 --pmc)")
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    cfg = list(CONFIGS[args.config])
    if args.batch:
        cfg[4] = args.batch
    cfg = tuple(cfg)
    arch, z, C, hw, B, mode, nl, hp, est = cfg

    torch.manual_seed(0)
    tr = make_trainer(cfg, device)
    from cvhip.engine import ClearStep

    eng = ClearStep.build(tr, mode)
    assert eng is not None, "fused engine unavailable"
    # synthetic batches resident in HBM before timing (distinct per rank)
    g = torch.Generator(device=device).manual_seed(1000 + rank)
    nb = 8
    Xs = [torch.rand(B, C, hw, hw, generator=g, device=device) for _ in range(nb)]
    Ls = [torch.randint(0, nl, (B,), generator=g, device=device) for _ in range(nb)]

    def step(i):
        out = eng.step(Xs[i % nb], Ls[i % nb])
        tr.annealer.step()
        return out

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if args.only_call:
        from cvhip import _lib

        G = eng.graphs[B]
        pname, idx = args.only_call.split("[")
        name, fn, cargs, _lane = G[pname].calls[int(idx.rstrip("]"))]
        s_ = _lib.stream_handle()
        for _ in range(args.reps):
            _lib.check(fn(*cargs, s_), name)
        torch.cuda.synchronize()
        print(json.dumps({"only_call": args.only_call, "name": name, "reps": args.reps}))
        return
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    losses = eng.last_workspace(B).losses if mode == "clear" else eng.last_workspace(B).losses
    finite = bool(torch.isfinite(losses[:4]).all())
    eng.sync_host_state()

    roof = None
    if not args.no_kernel_pass:
        G = eng.graphs[B]
        km = kernel_pass(eng, G)
        best = None
        for label, ms in km.items():
            fl = gemm_flops_of(label, G, eng)
            if fl is None:
                continue
            if best is None or ms > best[1]:
                best = (label, ms, fl)
        if best is not None:
            label, ms, fl = best
            ach = fl / (ms * 1e-3) / 1e12
            peak = PEAK_BF16_TFLOPS if hp.get("precision") == "bf16" else PEAK_FP32_TFLOPS
            roof = {"bound": "mfma", "kernel": label, "achieved": round(ach, 3), "peak": peak,
                    "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": None,
                    "kernel_ms": round(ms, 5), "flops_per_launch": fl}
            # HBM bytes per launch of the same call from the committed rocprofv3 PMC passes
            # (profiles/pmc_traffic.py), when they were taken on this call
            tpath = os.path.join(ROOT, "profiles", f"{args.config}_traffic.json")
            if os.path.exists(tpath):
                try:
                    t = json.load(open(tpath))["calls"].get(label.split(":")[0])
                    if t is not None:
                        roof["traffic"] = round(float(t["traffic_bytes"]))
                except (OSError, ValueError, KeyError):
                    pass
        step_ms_eager = sum(km.values())
        if args.kernel_table and rank == 0:
            with open(args.kernel_table, "w") as fh:
                fh.write(f"{'call':60s} {'ms':>9s} {'GFLOP':>9s} {'TF/s':>8s}\n")
                for label, ms in sorted(km.items(), key=lambda kv: -kv[1]):
                    fl = gemm_flops_of(label, G, eng)
                    fh.write(f"{label:60s} {ms:9.4f} {(fl or 0) / 1e9:9.3f} "
                             f"{(fl or 0) / (ms * 1e-3) / 1e12:8.2f}\n")
                fh.write(f"{'total':60s} {step_ms_eager:9.4f}\n")
    else:
        step_ms_eager = None

    if rank == 0:
        value = world * B * args.steps / el
        rec = {
            "metric": "training images/sec at bs=512; ELBO rel-err vs CPU ref",
            "value": round(value, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": hp.get("precision", "fp32"),
            "data": "synthetic U[0,1) images, uniform labels, resident in HBM; deterministic random-init weights",
            "config": {"workload": f"{args.config}: CLEAR-{'VAE' if mode == 'clear' else 'MIM (CLUB-S)'} {arch} "
                                   f"z={z} {C}x{hw}x{hw} per-GPU bs={B}", "model": arch, "global_batch": world * B,
                       "seq_len": None, "parallelism": f"dp{world}"},
            "algorithmic_tflops": round(conv_flops_per_image(eng.spec) * value / 1e12, 3),
            "losses_finite": finite,
            "roofline": roof,
            "eager_kernel_sum_ms": round(step_ms_eager, 4) if step_ms_eager else None,
        }
        if not args.no_cpu_baseline and world == 1:
            try:
                rec["cpu_baseline"] = cpu_baseline(cfg)
            except Exception as e:  # pragma: no cover
                rec["cpu_baseline"] = {"error": repr(e)}
            try:
                rec["elbo_rel_err"] = elbo_rel_err(cfg, device)
            except Exception as e:  # pragma: no cover
                rec["elbo_rel_err"] = repr(e)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
