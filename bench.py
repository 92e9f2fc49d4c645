"""CLEAR-VAE training throughput on MI355X (BASELINE.json metric: "training images/sec at bs=512;
ELBO rel-err vs CPU ref").

Default workload (configs[1]): Styled-MNIST-shaped synthetic batches [512, 1, 28, 28] ~ U[0,1), 10
labels, CLEAR-VAE (VAE, z=16, beta=1/8, lr 5e-4, alpha=100, tau=0.1, ps=True,
code/run_styledmnist_downstream_expr.py:231-238), fp32, one fused HIP training step per batch
(forward, ELBO, 2 contrastive terms, backward, Adam) through CLEARVAETrainer's engine.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config mnist|celeba-mim|celeba|camelyon-bf16]

--gpus N > 1: one process per GPU over RCCL.  Run directly, bench.py starts `torch.distributed.run
--nproc-per-node N` as a child process (before any GPU call) and passes its exit status on; under an
external torch.distributed.run WORLD_SIZE must equal N.  Per-GPU batch fixed (weak scaling); value = images
processed by all ranks / max-over-ranks wall time.  CV_DIST_BACKEND=gloo rehearses the flow with all ranks on
one GPU.  The default config also times, at every N, the weak-scaling keys "celeba" (VAE64 CLEAR-VAE fp32,
256 per GPU: north_star's scaling target), "pacs" (32 per GPU: configs[3] at N=4) and "camelyon_bf16" (128
per GPU bf16: configs[4] at N=8), each with the exposed all-reduce time per step at N > 1.

After the timed region (nothing below is inside it):
  (1) an in-step pass: the step's programs are enqueued eagerly behind a spin kernel long enough for the
      host to queue the whole step, with a HIP timing-event pair around every call on the step's stream
      (single-stream schedule), so each call's time is its duration inside a real step; the roofline is
      priced on the GEMM call with the largest in-step time (`roofline.kernel`), with HBM `traffic` from
      the committed rocprofv3 PMC passes of that call;
  (2) on rank 0 at N=1: the CPU baseline (oracle/ref_loop.py, the reference's step composition on
      torch-CPU) on a bounded sample, and the ELBO (and, for CLEAR-MIM, MI) error of one HIP step against
      the fp64 CPU reference on the same batch / weights / noise;
  (3) default config at N=1: configs[2] (CelebA 64x64 bs=256 CLEAR-MIM CLUB-S) is timed the same way
      and reported under "c3" with its own CPU baseline; the weak-scaling keys above at N=1 carry the
      in-step roofline of their dominant call ("c4_per_gpu" / "c5_per_gpu" repeat "pacs" /
      "camelyon_bf16", the round-2 names);
  (4) default / camelyon-bf16 config at N=1: the device input pipeline (Resize((64, 64)) + ToTensor of a
      96x96x3 uint8 batch of 1024, cv_load_batch_u8) under "input_pipeline", with Pillow's own transform
      timed beside it on one host core.
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
    # configs[3]: PACS resized to 64x64 before the model (code/run_pacs_downstream_expr.py:88-98), bs=128
    # over 4 GPUs = 32 per GPU, fp32; 7 domains' labels
    "pacs": ("VAE64", 64, 3, 64, 32, "clear", 7,
             dict(beta=1 / 32, vae_lr=3e-5, alpha=100.0, temperature=0.1, ps=True), None),
    # configs[4]: Camelyon17 patches resized to 64x64 before the model, bs=1024 over 8 GPUs =
    # 128 per GPU, bf16 contractions
    "camelyon-bf16": ("VAE64", 64, 3, 64, 128, "clear", 2,
                      dict(beta=1 / 32, vae_lr=3e-5, alpha=100.0, temperature=0.1, ps=True, precision="bf16"), None),
    # the same shard in fp32: the bf16 speed-up is measured in the same run (key camelyon_fp32, N = 1 only)
    "camelyon-fp32": ("VAE64", 64, 3, 64, 128, "clear", 2,
                      dict(beta=1 / 32, vae_lr=3e-5, alpha=100.0, temperature=0.1, ps=True), None),
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


def layer_flops(spec):
    """Algorithmic FLOPs of one forward pass per image (conv / linear MAC x 2)."""
    f = 0
    for c in spec.enc + spec.dec:
        k = c.mod.kernel_size[0] * c.mod.kernel_size[1]
        if c.transposed:
            macs = c.h_in * c.w_in * c.c_in * c.c_out * k
        else:
            macs = c.h_out * c.w_out * c.c_out * c.c_in * k
        f += 2 * macs
    f += 2 * spec.F * 4 * spec.d + 2 * 2 * spec.d * spec.dec_lin.out_features
    return f


def step_flops_per_image(spec, mode):
    """training = 3x forward; CLEAR-MIM adds 5 forward-only passes (the reference's work)."""
    f = layer_flops(spec)
    return 3 * f + (5 * f if mode == "mim" else 0)


def encoder_flops(spec):
    """Forward FLOPs per image of the encoder convs and the 4 heads."""
    f = 0
    for c in spec.enc:
        f += 2 * c.h_out * c.w_out * c.c_out * c.c_in * c.mod.kernel_size[0] * c.mod.kernel_size[1]
    return f + 2 * spec.F * 4 * spec.d


def executed_flops_per_image(spec, mode):
    """FLOPs the fused step executes per image: CLEAR-MIM's 5 estimator-update forwards share one encoder pass
    (same batch, same post-Adam weights: cvhip/engine.py make_learn), so 4 encoder passes are not run."""
    f = step_flops_per_image(spec, mode)
    return f - (4 * encoder_flops(spec) if mode == "mim" else 0)


def _programs(G):
    progs = [("fwd", G["fwd"]), ("dec", G["dec"]), ("lat", G["lat"]), ("enc", G["enc"])]
    if G.get("enc2") is not None:  # data parallel: the shallow-encoder bucket's program
        progs.append(("enc2", G["enc2"]))
    progs.append(("upd", G["upd"]))
    learn = G.get("learn")
    if isinstance(learn, list):  # data-parallel CLEAR-MIM: (gradient, Adam) program pairs
        for j, (gp, ap) in enumerate(learn):
            progs += [(f"learn{j}g", gp), (f"learn{j}a", ap)]
    elif learn is not None:
        progs.append(("learn", learn))
    return progs


def instep_pass(engine, G, rounds=6):
    """In-step device time of every call of the step program (see the module docstring): returns
    {label: mean ms per step} over `rounds` instrumented eager steps (a first one is discarded)."""
    names = {id(P): name for name, P in _programs(G)}
    segs = engine._segments(G, False)
    ncalls = sum(len(P.calls) for item in segs if item[0] == "prog" for P in item[1])
    acc, cnt = {}, 0
    for r in range(rounds + 1):
        torch.cuda.synchronize()
        torch.cuda._sleep(int(ncalls * 200_000))  # ~80 us of queue per call at ~2.4 GHz
        timers = []
        for item in segs:
            if item[0] == "prog":
                for P in item[1]:
                    t = []
                    P.run(timer=t)
                    timers.append((names[id(P)], P, t))
            elif item[0] == "ar":
                engine.buckets.launch(item[1])
            elif item[0] == "wait":
                engine.buckets.wait()
            elif item[0] == "ar_est":
                engine.est_buckets.launch(0)
            elif item[0] == "wait_est":
                engine.est_buckets.wait()
        torch.cuda.synchronize()
        if r == 0:
            continue
        cnt += 1
        for pname, P, t in timers:
            for i, e0, e1 in t:
                lab = f"{pname}[{i}]:{P.calls[i][0]}"
                acc[lab] = acc.get(lab, 0.0) + e0.elapsed_time(e1)
    return {k: v / cnt for k, v in acc.items()}


def isolated_pass(G, reps=20, rounds=3):
    """Per-call device time in isolation: each call captured REPS times back to back into its own HIP
    graph, replayed between HIP events.  (Repeating a call perturbs the workspace; run after timing.)"""
    from cvhip import _lib

    times = {}
    for pname, P in _programs(G):
        for i, (name, fn, args, _lane) in enumerate(P.calls):
            if (fn is None or _lane in ("join", "host")
                    or name in ("cv_ntxent_aux_combine", "cv_ntxent_aux_flush")):  # (a join; part of a queued phase)
                continue
            # a queued NT-Xent phase is timed on its own: queued (with the combine block attached to it, if the
            # program attaches one) and launched by a flush, as a step issues it when no launch serves it
            comb = None
            if name == "cv_ntxent_aux" and i + 1 < len(P.calls) and P.calls[i + 1][0] == "cv_ntxent_aux_combine":
                comb = P.calls[i + 1]
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                s = _lib.stream_handle()
                for _ in range(reps):
                    _lib.check(fn(*args, s), name)
                    if name == "cv_ntxent_aux":
                        if comb is not None:
                            _lib.check(comb[1](*comb[2], s), comb[0])
                        _lib.check(_lib.lib().cv_ntxent_aux_flush(s), "cv_ntxent_aux_flush")
                if name.endswith("_side"):  # (its weight gradient ran on a side stream: joined into the capture)
                    _join_side(args[-1])
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


def _join_side(handle):
    """The current stream waits for the side stream `handle` (a call that put work there, *_side)."""
    e = torch.cuda.Event()
    e.record(torch.cuda.ExternalStream(handle))
    torch.cuda.current_stream().wait_event(e)


def gemm_flops_of(label, G):
    """Algorithmic FLOPs of one conv / linear call from its program position (None for other calls)."""
    pname, rest = label.split("[", 1)
    idx = int(rest.split("]")[0])
    P = dict(_programs(G)).get(pname)
    if P is None:
        return None
    name, fn, args, _lane = P.calls[idx]
    # one contraction of the conv geometry: forward, backward-data or weight gradient (the `_kpack` entries carry
    # the other weight packing too; cv_convt_output_loss is the last ConvTranspose2d with the loss fused in)
    one = ("cv_conv_forward", "cv_conv_forward_kpack", "cv_convt_output_loss", "cv_conv_backward_data",
           "cv_conv_backward_data_kpack", "cv_conv_backward_weight", "cv_conv_backward_weight_deferred")
    two = ("cv_conv_backward_deferred", "cv_conv_backward_deferred_kpack",  # backward-data + weight gradient
           "cv_conv_backward_deferred_kpack_side")
    if name in one or name in two:
        g = args[0]._obj
        k = g.kh * g.kw
        if g.transposed:
            macs = g.n * g.h_in * g.w_in * g.c_in * g.c_out * k
        else:
            macs = g.n * g.h_out * g.w_out * g.c_out * g.c_in * k
        return 2.0 * macs * (2 if name in two else 1)
    if name in ("cv_linear_forward", "cv_linear_backward_data", "cv_linear_backward_weight"):
        g = args[0]._obj
        return 2.0 * g.n * g.in_features * g.out_features
    return None


def _one_stream(call):
    """A step-program call with its side-stream part on the call's own stream: cv_conv_backward_deferred_kpack_side
    as cv_conv_backward_deferred_kpack (the same kernels, back to back), so a prefix is one stream's chain and the
    difference of two prefixes is the call's own time, not the side stream's backlog."""
    name, fn, args, lane = call
    if name == "cv_conv_backward_deferred_kpack_side":
        from cvhip import _lib

        return (name[:-5], getattr(_lib.lib(), name[:-5]), list(args[:-1]), lane)
    return call


def prefix_times(engine, G, labels, reps=20, rounds=3):
    """In-graph, in-step duration of the given calls: a graph of the step's calls up to and including call
    i, minus one up to call i-1, each replayed REPS times between HIP events on the launch stream (min of
    ROUNDS).  The step's main-lane calls only (data parallel: the side-lane weight-gradient calls and the
    collectives between segments are left out, so a prefix is the single-stream chain the call runs in; a call
    that puts its weight gradient on side stream 1 runs both launches on the stream here, _one_stream);
    labels on a side lane are not timed.  Mutates the workspace (run after timing)."""
    from cvhip.plan import Program

    flat = []  # (label, call) in step order, main lane
    for pname, P in _programs(G):
        for i, c in enumerate(P.calls):
            if not c[3]:
                flat.append((f"{pname}[{i}]:{c[0]}", c))
    pos = {lab: k for k, (lab, _) in enumerate(flat)}
    labels = [lab for lab in labels if lab in pos]

    def t_prefix(k):
        if k < 0:
            return 0.0
        P = Program()
        P.calls = [_one_stream(c) for _, c in flat[:k + 1]]
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            P.run()
        g.replay()
        torch.cuda.synchronize()
        best = None
        for _ in range(rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            best = ms if best is None else min(best, ms)
        del g
        return best

    out = {}
    for lab in labels:
        k = pos[lab]
        out[lab] = t_prefix(k) - t_prefix(k - 1)
    return out


def roofline_of(config, G, instep, precision, engine=None, world=1):
    """Roofline of the GEMM call with the largest in-step time.  Candidates are ranked by the eager
    in-step pass (whose event pairs add a few us per call); the top three are then re-timed inside a
    replayed graph of the step by prefix differences (prefix_times), and the largest wins."""
    cands = []
    for label, ms in instep.items():
        fl = gemm_flops_of(label, G)
        if fl is not None:
            cands.append((ms, label, fl))
    if not cands:
        return None
    cands.sort(reverse=True)
    timing = "in-step HIP events on the call's stream (eager, event pairs per call)"
    if engine is not None:
        pt = prefix_times(engine, G, [lab for _, lab, _ in cands[:3]])
        if pt:  # (the main-lane calls among the top three)
            cands = sorted(((pt[lab], lab, fl) for _, lab, fl in cands[:3] if lab in pt), reverse=True)
            timing = "in-step, replayed step graph: t(prefix through the call) - t(prefix before it)"
    ms, label, fl = cands[0]
    best = (label, ms, fl)
    label, ms, fl = best
    ach = fl / (ms * 1e-3) / 1e12
    peak = PEAK_BF16_TFLOPS if precision == "bf16" else PEAK_FP32_TFLOPS
    roof = {"bound": "mfma", "kernel": label, "achieved": round(ach, 3), "peak": peak, "unit": "TFLOP/s",
            "frac": round(ach / peak, 4), "traffic": None, "kernel_ms": round(ms, 5), "flops_per_launch": fl,
            "timing": timing}
    # the kernels this call really issues (cv_debug_kernel_log around one more eager launch of it): a PMC figure
    # below is attached only if it was taken on exactly these kernels
    ran = call_kernels(G, label) if engine is not None and world == 1 else None
    if ran is not None:
        roof["kernels"] = ran
    # HBM bytes per launch of the same call from the committed rocprofv3 PMC passes
    # (profiles/pmc_traffic.py), when they were taken on this call (single-GPU programs: a data-parallel step's
    # program labels index a different call list, so N > 1 keys carry no PMC figures)
    tpath = os.path.join(ROOT, "profiles", f"{config}_traffic.json")
    if world > 1:
        return roof
    stale = {}
    if os.path.exists(tpath):
        try:
            t = json.load(open(tpath))["calls"].get(label)  # full "prog[i]:function" label of this build
            if t is not None:
                if ran is not None and _knorm(t.get("kernels", [])) != _knorm(ran):
                    stale["traffic_kernels"] = t.get("kernels", [])
                else:
                    roof["traffic"] = round(float(t["traffic_bytes"]))
        except (OSError, ValueError, KeyError):
            pass
    # MFMA utilisation of the same call from the committed counter pass (profiles/pmc_mfma.py), when taken
    upath = os.path.join(ROOT, "profiles", "mfma_util.jsonl")
    if os.path.exists(upath):
        try:
            key = f"{config} {label.split(':', 1)[0]}"
            for line in open(upath):  # (the last entry of a key wins)
                u = json.loads(line).get(key)
                if u is None:
                    continue
                if ran is not None and _knorm(u.get("kernels", [])) != _knorm(ran):
                    stale["mfma_util_kernels"] = u.get("kernels", [])
                    roof.pop("mfma_util_pmc", None)
                else:
                    stale.pop("mfma_util_kernels", None)
                    roof["mfma_util_pmc"] = round(float(u["mfma_util_median"]), 4)
        except (OSError, ValueError, KeyError):
            pass
    if stale:  # (refused: the committed counters describe other kernels than the ones timed)
        roof["pmc_refused"] = stale
    return roof


def _knorm(names):
    """Kernel names without return type, parameter list and spaces (rocprofv3 and __cxa_demangle spell them alike,
    up to whitespace)."""
    out = []
    for n in names:
        n = n.strip()
        if n.startswith("void "):
            n = n[5:]
        if n.endswith(")") and "(" in n:
            n = n[:n.rindex("(")]
        out.append(n.replace(" ", ""))
    return out


def call_kernels(G, label):
    """Demangled names of the kernels one eager launch of the step-program call `label` issues (mutates the
    workspace: run after timing)."""
    import ctypes

    from cvhip import _lib

    pname, rest = label.split("[", 1)
    P = dict(_programs(G)).get(pname)
    if P is None:
        return None
    idx = int(rest.split("]")[0])
    name, fn, cargs, _lane = P.calls[idx]
    # the NT-Xent phase queued right before the call (and its attached combine block) is queued again, so a launch
    # that serves it in the step logs the merged kernel it runs there; a phase it does not serve is dropped unlaunched
    pre = []
    j = idx - 1
    while j >= 0 and P.calls[j][0] in ("cv_ntxent_aux", "cv_ntxent_aux_combine"):
        pre.insert(0, P.calls[j])
        j -= 1
    L = _lib.lib()
    torch.cuda.synchronize()
    prev = L.cv_debug_kernel_log(1)
    try:
        s = _lib.stream_handle()
        for pn, pf, pa, _pl in pre:
            _lib.check(pf(*pa, s), pn)
        _lib.check(fn(*cargs, s), name)
        L.cv_ntxent_aux_discard()
        torch.cuda.synchronize()
        buf = ctypes.create_string_buffer(1 << 16)
        n = L.cv_debug_kernel_names(buf, len(buf))
    finally:
        L.cv_debug_kernel_log(prev)
    names = buf.value.decode().split("\n") if n else []
    return names


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg, budget_s=15.0):
    """The reference's training loop composition on the host cores (oracle/ref_loop.py, torch-CPU fp32),
    on a bounded sample of the same workload.  The host cores of the GPU boxes are shared, so single steps
    vary run to run: the value is the batch over the MEDIAN step time of the sample (mean and spread
    reported beside it), with the threads and the CPU affinity used."""
    import statistics

    from oracle.ref_loop import RefLoop

    arch, z, C, hw, B, mode, nl, hp, est = cfg
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):  # pragma: no cover
        affinity = os.cpu_count() or 1
    threads = int(os.environ.get("OMP_NUM_THREADS", affinity))
    torch.set_num_threads(threads)
    loop = RefLoop(arch, z, C, mode, dict(hp))
    g = torch.Generator().manual_seed(1000)
    data = [(torch.rand(B, C, hw, hw, generator=g), torch.randint(0, nl, (B,), generator=g)) for _ in range(4)]
    loop.step(*data[0])  # warm-up (allocator, oneDNN primitives)
    times = []
    while sum(times) < budget_s and len(times) < 400:
        X, y = data[len(times) % len(data)]
        t0 = time.perf_counter()
        loop.step(X, y)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    kind = "CLEAR-VAE" if mode == "clear" else "CLEAR-MIM CLUB-S"
    return {"value": round(B / med, 1), "unit": "images/s", "cores": torch.get_num_threads(),
            "cpu_affinity": affinity, "cpu_model": cpu_model(), "kind": "port",
            "mean_value": round(B * len(times) / sum(times), 1),
            "step_ms_p10_p50_p90": [round(1e3 * statistics.quantiles(times, n=10)[0], 2) if len(times) > 1 else None,
                                    round(1e3 * med, 2),
                                    round(1e3 * statistics.quantiles(times, n=10)[-1], 2) if len(times) > 1 else None],
            "sample": f"{len(times)} steps x bs={B} {arch} {kind} fp32 (median step): "
                      "oracle/ref_loop.py, the reference's module/loss/trainer step composition on torch-CPU "
                      "(within 1% of the reference's own _train in the dev container, DESIGN 7)"}


def step_error(cfg, device):
    """One fused HIP step on a fixed batch with injected noise (and CLUB-S permutation) vs the fp64 CPU
    reference: relative ELBO error (rec + w*KL_c + w*KL_s) and, for CLEAR-MIM, the MI error with an
    absolute floor (|d| / max(|mi|, 1))."""
    import numpy as np

    from cvhip import rng
    from cvhip.engine import ClearStep
    from oracle import cpu_ref as R

    arch, z, C, hw, B, mode, nl, hp, est = cfg
    tr = make_trainer(cfg, device)
    sd = R.det_state(arch, z, C)
    tr.model.load_state_dict({k: torch.as_tensor(np.asarray(v)).float() if np.asarray(v).dtype != np.int64
                              else torch.as_tensor(np.asarray(v)) for k, v in sd.items()})
    x, label, ec, es, perm = R.det_inputs(B, C, hw, z, nl, seed=77)
    rng.clear_injections()
    X = torch.tensor(x, dtype=torch.float32, device=device)
    L = torch.tensor(label, device=device)
    w = R.anneal_weight(0, hp["beta"])
    if mode == "clear":
        eng = ClearStep.build(tr, "clear")
        rng.inject_noise([torch.tensor(ec, dtype=torch.float32), torch.tensor(es, dtype=torch.float32)])
        Lh = eng.step(X, L).cpu()
        hpp = dict(temperature=hp["temperature"], alpha=hp["alpha"], beta=hp["beta"], ps=hp["ps"])
        o = R.clear_step(R.to_torch(sd), torch.tensor(x), torch.tensor(label), torch.tensor(ec), torch.tensor(es),
                         arch, hpp)
        out = {}
    else:
        M = R.det_mlp(z // 2, z)
        tr.mi_estimator.load_state_dict({k: torch.tensor(v, dtype=torch.float32) for k, v in M.items()})
        eng = ClearStep.build(tr, "mim")
        gen = np.random.default_rng(5)
        noise = [ec, es] + [gen.standard_normal((B, z // 2)) for _ in range(10)]
        rng.inject_noise([torch.tensor(a, dtype=torch.float32) for a in noise])
        rng.inject_perm([torch.tensor(perm)])
        Lh, _ = eng.step(X, L)
        Lh = Lh.cpu()
        hpp = dict(temperature=hp["temperature"], alpha=hp["alpha"], beta=hp["beta"], **{"lambda": hp["la"]})
        o = R.mim_step(R.to_torch(sd), R.to_torch(M), torch.tensor(x), torch.tensor(label), torch.tensor(ec),
                       torch.tensor(es), torch.tensor(perm), arch, hpp, est)
        mi_ref = float(o["mi"].detach())
        out = {"mi_abs_err": abs(float(Lh[5]) - mi_ref), "mi_rel_err": abs(float(Lh[5]) - mi_ref) / max(abs(mi_ref), 1.0)}
    elbo_hip = float(Lh[0]) + w * float(Lh[1]) + w * float(Lh[2])
    elbo_ref = float(o["rec"].detach()) + w * float(o["kl_c"].detach()) + w * float(o["kl_s"].detach())
    out["elbo_rel_err"] = abs(elbo_hip - elbo_ref) / abs(elbo_ref)
    return out


def run_workload(name, cfg, steps, warmup, device, world, rank, detail=True, kernel_table=None):
    """Time `steps` fused steps of configuration `cfg` (after `warmup`), then the in-step pass."""
    from cvhip.engine import ClearStep

    arch, z, C, hw, B, mode, nl, hp, est = cfg
    torch.manual_seed(0)
    tr = make_trainer(cfg, device)
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

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    finite = bool(torch.isfinite(eng.last_workspace(B).losses[:4]).all())
    eng.sync_host_state()
    value = world * B * steps / max(el, 1e-12)
    res = {"value": value, "el": el, "ms_per_step": el / max(steps, 1) * 1e3, "finite": finite, "eng": eng,
           "algorithmic_tflops": step_flops_per_image(eng.spec, mode) * value / 1e12,
           "executed_tflops": executed_flops_per_image(eng.spec, mode) * value / 1e12}
    if world > 1:
        res["comm"] = comm_pass(eng, step, warmup + steps, device)
    if detail:
        G = eng.graphs[B]
        instep = instep_pass(eng, G)
        res["instep"] = instep
        res["roofline"] = roofline_of(name, G, instep, hp.get("precision", "fp32"), eng, world)
        res["instep_sum_ms"] = sum(instep.values())
        if kernel_table and rank == 0:
            iso = isolated_pass(G)
            with open(kernel_table, "w") as fh:
                fh.write(f"{'call':60s} {'in-step ms':>11s} {'isolated':>9s} {'GFLOP':>8s} {'TF/s in-step':>12s}\n")
                for label, ms in sorted(instep.items(), key=lambda kv: -kv[1]):
                    fl = gemm_flops_of(label, G) or 0
                    fh.write(f"{label:60s} {ms:11.4f} {iso.get(label, 0):9.4f} {fl / 1e9:8.3f} "
                             f"{fl / (ms * 1e-3) / 1e12:12.2f}\n")
                fh.write(f"{'total (sum of calls)':60s} {sum(instep.values()):11.4f} {sum(iso.values()):9.4f}\n")
    return res


def comm_pass(eng, step, i0, device, k=10):
    """Data parallel: the exposed (not overlapped) gradient all-reduce time per step, from HIP events around
    every wait for the buckets on the step's stream over K instrumented steps (after the timed region), max
    over ranks; with the bucket sizes."""
    eng.comm_probe = []
    torch.cuda.synchronize()
    for i in range(k):
        step(i0 + i)
    torch.cuda.synchronize()
    tot = {"vae": 0.0, "est": 0.0}
    for kind, e0, e1 in eng.comm_probe:
        tot[kind] += e0.elapsed_time(e1)
    eng.comm_probe = None
    t = torch.tensor([tot["vae"] / k, tot["est"] / k], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    out = {"exposed_allreduce_ms": round(float(t[0]), 4),
           "bucket_bytes": [4 * (hi - lo) for lo, hi in eng.buckets.bounds],
           "timing": "HIP events around the wait for the gradient buckets on the step stream, mean of "
                     f"{k} steps, max over ranks"}
    if eng.two_nets:
        out["exposed_estimator_allreduce_ms"] = round(float(t[1]), 4)
    return out


def pipeline_pass(device, n=1024, hw=96, out=64, reps=50, cpu_budget_s=3.0):
    """The device input pipeline (cv_load_batch_u8): Resize((64, 64)) + ToTensor of a
    Camelyon17-shaped batch (96x96x3 uint8 patches resident in HBM, random sample of a 4096-image set;
    configs[4]'s global batch 1024) timed with HIP events over `reps` back-to-back launches, priced on HBM
    bytes (uint8 in + fp32 out per image).  Beside it, the reference's own transform — Pillow
    Image.resize(BILINEAR) + ToTensor's /255, one image at a time on one host core, as its DataLoader
    (num_workers=0) runs it — on a bounded sample."""
    import numpy as np

    from cvhip.data import load_batch

    g = np.random.default_rng(0)
    imgs = torch.tensor(g.integers(0, 256, size=(4096, hw, hw, 3), dtype=np.uint8), device=device)
    idx = torch.tensor(g.integers(0, 4096, size=n), device=device)
    dst = torch.empty(n, 3, out, out, dtype=torch.float32, device=device)
    for _ in range(5):
        load_batch(imgs, idx, (out, out), out=dst, checked=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        load_batch(imgs, idx, (out, out), out=dst, checked=False)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000.0 / reps
    per_img = hw * hw * 3 + 3 * out * out * 4
    gbs = per_img * n / (us * 1e-6) / 1e9
    rec = {"op": f"Resize(({out},{out}))+ToTensor of {hw}x{hw}x3 uint8, gather by index (cv_load_batch_u8)",
           "batch": n, "us_per_batch": round(us, 2), "images_per_s": round(n / (us * 1e-6), 1),
           "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
                        "frac": round(gbs / PEAK_HBM_GBS, 4), "unit": "GB/s", "traffic": None,
                        "bytes_per_image": per_img}}
    # HBM bytes per launch from the committed PMC passes of the same launch (tools/pipe_pmc.py,
    # profiles/pmc_traffic.py): taken at this shape only
    try:
        t = json.load(open(os.path.join(ROOT, "profiles", "pipeline_traffic.json")))["calls"]
        if n == 1024 and hw == 96 and out == 64:
            rec["roofline"]["traffic"] = round(float(t["load_batch_u8:camelyon96_bs1024"]["traffic_bytes"]))
    except (OSError, ValueError, KeyError):
        pass
    try:
        from PIL import Image

        host = imgs[:256].cpu().numpy()
        t0, k = time.perf_counter(), 0
        while time.perf_counter() - t0 < cpu_budget_s:
            im = Image.fromarray(host[k % 256]).resize((out, out), Image.BILINEAR)
            np.asarray(im, dtype=np.float32).transpose(2, 0, 1) / np.float32(255)
            k += 1
        dt = time.perf_counter() - t0
        rec["cpu_reference"] = {"images_per_s": round(k / dt, 1), "cores": 1, "kind": "reference",
                                "sample": f"{k} images, Pillow Image.resize(BILINEAR) + /255, {dt:.1f} s"}
    except ImportError:  # pragma: no cover
        rec["cpu_reference"] = None
    return rec


def workload_label(name, cfg, world):
    arch, z, C, hw, B, mode, nl, hp, est = cfg
    kind = "CLEAR-VAE" if mode == "clear" else "CLEAR-MIM (CLUB-S)"
    return {"workload": f"{name}: {kind} {arch} z={z} {C}x{hw}x{hw} per-GPU bs={B} {hp.get('precision', 'fp32')}",
            "model": arch, "global_batch": world * B, "seq_len": None, "parallelism": f"dp{world}"}


def spawn_ranks(n):
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


# weak-scaling workloads timed at every N by the default run (per-GPU batch fixed): north_star's 75 % scaling
# target is on CelebA 64x64 (code/run_celeba_downstream_expr.py:225-234, VAE64 z=64 CLEAR-VAE, 256 per GPU);
# PACS 32 per GPU is configs[3] at N=4, Camelyon17 128 per GPU bf16 is configs[4] at N=8
SCALING_KEYS = (("celeba", "celeba", 256), ("pacs", "pacs", 32), ("camelyon_bf16", "camelyon-bf16", 128))


def scaling_entry(cname, cfg, steps, device, world, rank, detail):
    r = run_workload(cname, cfg, steps, 10, device, world, rank, detail=detail)
    e = {"value": round(r["value"], 1), "unit": "images/s", "n_gpus": world, "scaling": "weak",
         "per_gpu_batch": cfg[4], "global_batch": world * cfg[4], "ms_per_step": round(r["ms_per_step"], 4),
         "steps": steps, "dtype": cfg[7].get("precision", "fp32"), "config": workload_label(cname, cfg, world),
         "losses_finite": r["finite"], "algorithmic_tflops": round(r["algorithmic_tflops"], 3)}
    if "comm" in r:
        e.update(r["comm"])
    if r.get("roofline") is not None:
        e["roofline"] = r["roofline"]
    e["roofline_step"] = step_roofline(r["algorithmic_tflops"], world, cfg[7].get("precision", "fp32"))
    return e


def step_roofline(alg_tflops, world, precision):
    """Whole-step MFMA roofline of a key at N GPUs: the reference's algorithmic FLOP rate per GPU over the dense
    peak of the compute dtype (the dominant call's own roofline is `roofline`)."""
    peak = PEAK_BF16_TFLOPS if precision == "bf16" else PEAK_FP32_TFLOPS
    per = alg_tflops / max(world, 1)
    return {"bound": "mfma", "achieved_per_gpu": round(per, 3), "peak": peak, "unit": "TFLOP/s",
            "frac": round(per / peak, 4), "n_gpus": world}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="mnist", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-pass", action="store_true", help="skip the in-step pass (profiling runs)")
    ap.add_argument("--no-c3", action="store_true", help="default config: skip the configs[2] extra keys")
    ap.add_argument("--kernel-table", default=None, help="write the per-call timing table to this file")
    ap.add_argument("--only-call", default=None,
                    help="profiling mode: after warmup, launch this step-program call (e.g. 'enc[4]') --reps "
                         "times back to back and exit (for rocprofv3 --pmc)")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--list-calls", action="store_true",
                    help="print every step-program call label with the kernels one launch of it runs (profiling aid)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch check without a GPU: the ranks join a gloo group and rank 0 prints the world")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: start torch.distributed.run as a child process before anything touches the GPU
        # (this process never initialises HIP) and pass its exit status on; rank 0 prints the line
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (torch.distributed.run --nproc-per-node "
                 "must equal --gpus)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:  # (tests/test_bench_launch.py: the rank launch on a machine without a GPU)
        if world > 1:
            dist.init_process_group("gloo")
            t = torch.ones(1)
            dist.all_reduce(t)
            world_seen = int(t.item())
        else:
            world_seen = 1
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "world_seen": world_seen, "gpus_arg": args.gpus}),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    # RCCL over xGMI; CV_DIST_BACKEND=gloo rehearses the multi-rank flow with several ranks on one GPU
    backend = os.environ.get("CV_DIST_BACKEND", "nccl")
    if world > 1 and backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            from cvhip.dist import prepare_captured_collectives_env
            prepare_captured_collectives_env()
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    cfg = list(CONFIGS[args.config])
    if args.batch:
        cfg[4] = args.batch
    cfg = tuple(cfg)
    arch, z, C, hw, B, mode, nl, hp, est = cfg

    if args.only_call:
        from cvhip import _lib

        res = run_workload(args.config, cfg, 0, args.warmup, device, world, rank, detail=False)
        G = res["eng"].graphs[B]
        pname, idx = args.only_call.split("[")
        name, fn, cargs, _lane = dict(_programs(G))[pname].calls[int(idx.rstrip("]"))]
        s_ = _lib.stream_handle()
        for _ in range(args.reps):
            _lib.check(fn(*cargs, s_), name)
        torch.cuda.synchronize()
        print(json.dumps({"only_call": args.only_call, "name": name, "reps": args.reps}))
        return

    if args.list_calls:  # (each call launched once more, eagerly: mutates the workspace)
        res = run_workload(args.config, cfg, 0, args.warmup, device, world, rank, detail=False)
        G = res["eng"].graphs[B]
        for pname, P in _programs(G):
            for i, c in enumerate(P.calls):
                if c[1] is None or c[3] in ("join", "host") or c[0].startswith("cv_ntxent_aux"):
                    continue
                label = f"{pname}[{i}]:{c[0]}"
                print(json.dumps({"label": label, "lane": c[3], "kernels": call_kernels(G, label)}))
        return

    res = run_workload(args.config, cfg, args.steps, args.warmup, device, world, rank,
                       detail=not args.no_kernel_pass, kernel_table=args.kernel_table)
    c3 = None
    extra = args.config == "mnist" and not args.no_c3 and args.batch is None
    if extra and world == 1:
        ccfg = CONFIGS["celeba-mim"]
        k3 = min(args.steps, 60)
        r3 = run_workload("celeba-mim", ccfg, k3, 5, device, 1, 0, detail=not args.no_kernel_pass)
        c3 = {"metric": "training images/sec (configs[2])", "value": round(r3["value"], 1), "unit": "images/s",
              "ms_per_step": round(r3["ms_per_step"], 4), "steps": k3, "warmup": 5, "dtype": "fp32",
              "config": workload_label("celeba-mim", ccfg, 1),
              "algorithmic_tflops": round(r3["algorithmic_tflops"], 3),
              "algorithmic_tflops_note": "the reference's work (6 VAE forwards per step, SURVEY 8d)",
              "executed_tflops": round(r3["executed_tflops"], 3),
              "executed_tflops_note": "the work run: the 5 estimator-update forwards share one encoder pass",
              "losses_finite": r3["finite"], "roofline": r3.get("roofline")}
    # the weak-scaling keys at every N (per-GPU batch fixed; at N=1 the same workloads on one GPU, with the
    # in-step roofline of their dominant call)
    scaling = {}
    if extra:
        for key, cname, bs in SCALING_KEYS:
            ccfg = CONFIGS[cname]
            assert ccfg[4] == bs, (cname, ccfg[4])
            scaling[key] = scaling_entry(cname, ccfg, min(args.steps, 100), device, world, rank,
                                         detail=not args.no_kernel_pass)
        if world == 1:  # (configs[4]'s shard in fp32 beside the bf16 key: their ratio is the bf16 speed-up)
            scaling["camelyon_fp32"] = scaling_entry("camelyon-fp32", CONFIGS["camelyon-fp32"], min(args.steps, 100),
                                                     device, world, rank, detail=False)
            scaling["camelyon_bf16"]["speedup_vs_fp32"] = round(scaling["camelyon_bf16"]["value"]
                                                                / scaling["camelyon_fp32"]["value"], 4)
    if rank == 0:
        rec = {
            "metric": "training images/sec at bs=512; ELBO rel-err vs CPU ref",
            "value": round(res["value"], 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(res["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": hp.get("precision", "fp32"),
            "data": "synthetic U[0,1) images, uniform labels, resident in HBM; deterministic random-init weights",
            "config": workload_label(args.config, cfg, world),
            "algorithmic_tflops": round(res["algorithmic_tflops"], 3),
            "losses_finite": res["finite"],
            "roofline": res.get("roofline"),
            "roofline_step": step_roofline(res["algorithmic_tflops"], world, hp.get("precision", "fp32")),
            "instep_sum_ms": round(res["instep_sum_ms"], 4) if "instep_sum_ms" in res else None,
        }
        if "comm" in res:
            rec.update(res["comm"])
        rec.update(scaling)
        if world == 1 and scaling:  # (the round-2 names of the configs[3] / configs[4] per-GPU shards)
            rec["c4_per_gpu"] = scaling["pacs"]
            rec["c5_per_gpu"] = scaling["camelyon_bf16"]
        if world == 1:
            try:
                rec.update(step_error(cfg, device))
            except Exception as e:  # pragma: no cover
                rec["elbo_rel_err"] = repr(e)
            if c3 is not None:
                try:
                    c3.update(step_error(CONFIGS["celeba-mim"], device))
                except Exception as e:  # pragma: no cover
                    c3["elbo_rel_err"] = repr(e)
                if not args.no_cpu_baseline:
                    try:
                        c3["cpu_baseline"] = cpu_baseline(CONFIGS["celeba-mim"], budget_s=12.0)
                    except Exception as e:  # pragma: no cover
                        c3["cpu_baseline"] = {"error": repr(e)}
                rec["c3"] = c3
            if args.config in ("mnist", "camelyon-bf16") and args.batch is None:
                try:
                    rec["input_pipeline"] = pipeline_pass(device)
                except Exception as e:  # pragma: no cover
                    rec["input_pipeline"] = {"error": repr(e)}
            if not args.no_cpu_baseline:
                try:
                    rec["cpu_baseline"] = cpu_baseline(cfg)
                except Exception as e:  # pragma: no cover
                    rec["cpu_baseline"] = {"error": repr(e)}
                if args.config == "mnist" and args.batch is None:
                    # BASELINE configs[0]: Styled-MNIST bs=64 CLEAR-VAE on the reference's CPU path
                    # (reference step: code/src/trainer.py:435-493), timed on the same host cores
                    try:
                        c1 = list(cfg)
                        c1[4] = 64
                        rec["cpu_baseline_c1"] = dict(cpu_baseline(tuple(c1), budget_s=8.0),
                                                      config="configs[0]: Styled-MNIST 28x28 bs=64 CLEAR-VAE, "
                                                             "reference CPU path (no GPU)")
                    except Exception as e:  # pragma: no cover
                        rec["cpu_baseline_c1"] = {"error": repr(e)}
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
