"""Fused CLEAR training step: one HIP program per step, replayed as a HIP graph.

ClearStep runs the body of CLEARVAETrainer._train (code/src/trainer.py:447-484) or of
ClearMIMVAETrainer._train (code/src/trainer.py:842-888) as a fixed sequence of libclearvae_hip.so
calls over device-resident buffers:

  zero(stats, grads) -> encoder (conv + fused BN/ReLU) -> heads -> reparam -> decoder -> output BN +
  sigmoid + reconstruction loss + backward seed -> decoder backward -> KL / contrastive / MI
  gradients into d(heads) -> heads + encoder backward -> BN affine grads -> [RCCL all-reduce] ->
  Adam on the flat parameter arena (+ LogisticAnnealer step on the device)

For CLEAR-MIM the 5 estimator updates follow (each: a train-mode forward for BN statistics and z,
then one fused learning-loss + Adam kernel on the estimator arena).  For the GVAE / ML-VAE baselines
(HierarchicalVAETrainer._train, code/src/trainer.py:326-353; mode "group") the reparameterisation is the
label-segmented group evidence (cv_group_forward: no host round trip for the groups) and the latent
terms are cv_group_backward (kl_c over the groups, the B/m adjustment of rec and kl_s).

The first step at a new batch size runs eagerly (it also loads the code objects); the second is
captured into a torch.cuda.CUDAGraph and every later step replays it.  Step-varying scalars (RNG
offset, Adam step, annealer step) live in device counters advanced by the kernels, so replays need
no host writes.  Host-visible PyTorch state (param .data / .grad, optimizer.state exp_avg /
exp_avg_sq, BN running stats) are views of, or are updated in place by, the same device buffers;
the optimizer's CPU 'step' counters are synchronised at the end of every epoch (sync_host_state).

Data parallel (cvhip/dist.py): when torch.distributed is initialised with world_size > 1, rank 0's
parameters are broadcast once, and each step is split into graph segments with the gradient
all-reduce (RCCL over xGMI, SUM, scaled by 1/world inside the Adam kernel) between them: the
decoder bucket is launched asynchronously as soon as the decoder backward segment has run, so it
overlaps the latent + encoder backward segment; the encoder bucket follows and the Adam segment
waits for both.  In CLEAR-MIM each of the 5 estimator updates all-reduces the estimator gradient
between its gradient and Adam segments.  Semantics are those of torch DDP around the reference
(local-batch BN / contrastive / MI terms, averaged gradients).
"""

from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from . import _lib, rng
from . import dist as cvdist
from ._lib import (GROUP, MI_CLUBSAMPLE, MI_L1OUT, SIM, cv_latent_chain, cv_mlp, cv_mlp_grad, cv_ntxent_branch,
                   cv_tc_disc, cv_tc_grad)
from .autograd import est_params, mlp_struct
from ._lib import cv_conv_pack
from .plan import (DeferGroup, ParamArena, Program, Workspace, ensure_arena, pack_program, ptr_array,
                   struct_array)


# CVHIP_FUSED_ADAM=1: single-process steps run the optimizer inside the end-of-backward reduction
# (cv_step_reduce_adam: one launch less, but the reduction's gradient order makes the Adam read-modify-writes
# strided; MNIST 777k vs 791k img/s, CelebA 99.7k vs 102.3k), so the separate cv_adam_step stays the default
FUSED_ADAM = os.environ.get("CVHIP_FUSED_ADAM", "0") == "1"  # measured slower (strided Adam RMW): off

# CVHIP_GRAPH_COLLECTIVES=1 (opt-in): a data-parallel step is captured as ONE graph with its RCCL all-reduces inside
# (issued on the capturing stream: the process group's collective stream joins the capture behind an event edge, the
# collective's branch runs beside the next backward segment and the Adam segment waits on it), so a step is one
# graph launch from the host instead of 4 launches + 3 all-reduce calls + 1 wait (CLEAR-MIM: + 5 x (launch,
# all-reduce, wait, launch)).  Off by default: it needs a backend that supports stream capture (RCCL; not gloo,
# which the world-2 tests use: ClearStep refuses it), and the one-GPU box can only rehearse it at world 1
# (tests/test_gpu_graph_collectives.py).  The bucket collectives then run on a dedicated RCCL group created with
# its CUDA-event cache off (cvhip.dist.captured_collectives_group), so no caller setup is needed.
GRAPH_COLLECTIVES = os.environ.get("CVHIP_GRAPH_COLLECTIVES", "0") == "1"

# CVHIP_LATENT_SIDE=1 (A/B knob, off: measured slower): the NT-Xent terms depend only on the heads, so their two launches (row
# log-sum-exps, then the gradients, accumulated into a d(heads) the step's first launch zeroed) fork onto a side
# stream right after the heads launch and run beside the decoder forward / backward; the step joins them before the
# KL / decoder-chain seed (cv_latent_combine_acc), which now adds onto them.  The same two adds per element, in the
# other order: d(heads) is bit-identical.  Single-graph steps only (a data-parallel step captured per segment would
# leave the fork unjoined in its first graph).  Measured (round 5, same box, 2 rounds): MNIST 0.5155 -> 0.5241 ms,
# C3 4.236 -> 4.276 ms — the graph's fork / join edges cost more than the 31 us of NT-Xent they take off the
# critical path, as for the side-stream weight gradients; so the two launches stay on the critical
# path (cv_latent_step).
LATENT_SIDE = os.environ.get("CVHIP_LATENT_SIDE", "0") == "1"

# CVHIP_LATENT_AUX (default 1): the NT-Xent phases queued into the decoder forward instead (cv_ntxent_aux): the row
# log-sum-exps ride in the first decoder ConvTranspose2d's grid, the losses and gradients (accumulated into the
# zeroed d(heads)) in the second's, as extra workgroups of the same launch where the library serves the pair
# (cv_aux.hip), else as their own launches at those points; the KL / decoder-chain seed adds onto them after the
# decoder backward (cv_latent_combine_acc).  One stream, no graph edges; d(heads) is bit-identical (the same two adds
# per element, in the other order).
LATENT_AUX = os.environ.get("CVHIP_LATENT_AUX", "1") == "1"
# CVHIP_LATENT_AUX_OUT=1 (A/B knob, off; with LATENT_AUX): the gradient phase is queued before the last decoder
# conv instead of the second: the output-loss launch that follows the image-side scatter serves it (cv_output_loss),
# and the second ConvTranspose2d's grid runs alone.  Measured (round 5, MNIST, two rounds): ConvT2 35.3 -> 27.5 us
# in-step but the output call 22.1 -> 31.4 us, step 0.4960 -> 0.4966 ms — the phase costs ~9 us wherever it rides.
LATENT_AUX_OUT = os.environ.get("CVHIP_LATENT_AUX_OUT", "0") == "1"

# CVHIP_LATENT_CHAIN=1 (A/B knob, off; with LATENT_AUX): the latent combine split at its dependency.  Its KL part (losses
# 1, 2, 7 and the KL gradient, written into the zeroed d(heads)) needs only the heads, so it rides as one more
# workgroup of the rows phase's grid (cv_ntxent_aux_combine); its decoder-chain part needs dz, which the decoder
# backward produces, and is added by the fused heads backward as it stages d(heads) (cv_heads_backward_chain, which
# also writes losses[0]).  The step loses the one-workgroup combine launch between the decoder and the encoder
# backward.  d(heads) in memory then holds the KL + contrastive (+ MI) terms only; the sums differ from the
# one-launch combine's by the order of two fp32 adds per element.  Opt-in (measured slower, round 5: MNIST 0.5025
# -> 0.5145 ms — the chain term's three extra operands cost the heads backward's staging 13.0 -> 22.3 us, more than
# the combine launch it replaces, and the KL workgroup lengthened the rows-phase grid by 12 us).
LATENT_CHAIN = os.environ.get("CVHIP_LATENT_CHAIN", "0") == "1"

# CVHIP_LATENT_AUX_DL (default 1; with LATENT_AUX, without LATENT_CHAIN / LATENT_AUX_OUT): the NT-Xent phases ride in
# the decoder-input launches instead of the decoder ConvTranspose2d grids: the row log-sum-exps in the decoder-input
# forward's grid, the losses and gradients in the decoder-input backward's (cv_declinear.hip
# declinear_*_aux_kernel).  Those grids hold 128 workgroups of 512 threads, so half the CUs are free for the phases;
# the ConvTranspose2d grids serve only d <= 8 (a larger register phase spills there).  Taken where those grids do not
# serve the phase (d > 8: every VAE64 config, register NT-Xent for d <= 32, n <= 256).  Measured (round 6, same box,
# two rounds): CelebA 2.1276 -> 2.0994 ms (the two standalone NT-Xent launches, 17 + 25 us, hidden in the decoder-input
# grids); on MNIST (d = 8) the ConvTranspose2d placement stays: there the phases cost ~2 us each, in the decoder-input
# grids 6 + 4 us (0.4735 -> 0.4820 ms with them there: CVHIP_LATENT_AUX_DL=2 forces it).
LATENT_AUX_DL = int(os.environ.get("CVHIP_LATENT_AUX_DL", "1"))

# CVHIP_ADAM_PACK (default auto: on for arenas of >= 2^20 parameters, i.e. VAE64; 1 / 0 force; single GPU and data
# parallel, not with CVHIP_FUSED_ADAM): the VAE's Adam step packs the
# conv weights it has just updated in the same launch (cv_adam_pack_step), so the packed copies are current when the
# next forward starts: a replayed step's first launch only zeroes (and copies the batch), and CLEAR-MIM's / CLEAR-TC's
# estimator forwards after the update need no packing launch.  Parameters changed outside the engine between steps
# (load_state_dict, torch optimizers, writes into the arena buffer: anything that bumps a parameter's or the arena's
# version counter) are repacked before the next replay; changes through a parameter's `.data` alias bypass the
# counters: call ClearStep.invalidate_packed() after them.
# Measured (same box, two rounds, after fixing the CVHIP_ADAM_PACK=0 programs, which had run the reduction and the
# optimizer twice): MNIST 0.4724 ms unfused vs 0.4842 fused, CelebA 1.8986 vs 1.8888 — the packing launch at the step
# start costs the small model less than the packing workgroups inside its Adam launch.
ADAM_PACK = os.environ.get("CVHIP_ADAM_PACK", "auto")
ADAM_PACK_MIN = 1 << 20

# CVHIP_DET_DZ (default 1; the LATENT_AUX / LATENT_SIDE schedules): the decoder-input gradient dz = d(h) W is computed
# by the latent combine launch (cv_latent_combine_dz, fixed-order sums) instead of as fp32-atomic partials in the
# decoder-input backward — the fused step's only order-dependent sum, so with it replays from the same state are
# bit-identical (tests/test_gpu_determinism.py); 0: the atomic partials (A/B)
DET_DZ = os.environ.get("CVHIP_DET_DZ", "1") == "1"

# CVHIP_MIM_BRANCHES (default 2; 0: the sequential form): CLEAR-MIM's five estimator-update decoder forwards
# (trainer.py:873-888) on this many side lanes of the single-GPU step graph, beside the five estimator learning steps
# on the step's stream (ClearStep._programs, make_learn_branched).  Measured (round 6, VAE64 n = 256, the five
# decoder forwards alone in a graph, scratch experiment): back to back 1.50 ms; on 5 / 3 / 2 lanes 1.23 / 1.20 /
# 1.25 ms; one decoder pass over 5 x 256 images (the bound of a segmented-statistics kernel) 1.27 ms.  In the step,
# with the side-stream weight gradients of the VAE step (WGRAD_LANE): 1 / 2 / 3 lanes 3.730 / 3.511 / 3.480 ms on one
# box (two rounds), 2 / 3 lanes 3.497 / 3.529 ms on another: 2 and 3 within the boxes' spread, 2 kept.
MIM_BRANCHES = int(os.environ.get("CVHIP_MIM_BRANCHES", "2"))

# CVHIP_PACK_COPY (default 1): a replayed step's first launch (weight packing + step zeroing) is issued eagerly before
# the step graph with the batch copy folded in (cv_pack_conv_weights_zero_copy); 0: the packing is the graph's first
# node and the copy a launch of its own (A/B)
PACK_COPY = os.environ.get("CVHIP_PACK_COPY", "1") == "1"

# CVHIP_WGRAD_LANE (default 2): the deferred weight gradients of the conv / convT layers off the image (the image-side
# layers keep their fused edge launches) on side stream 1 (Workspace.wgrad_side, cv_conv_backward_deferred_kpack_side):
# each runs beside its own and the next layers' backward-data launches instead of between them; every program joins
# the side stream before its cv_step_reduce (single process: once, in `enc`; data parallel: once per gradient bucket,
# so each graph segment ends joined).  Same box, two rounds: CelebA 2.089 -> 1.930 ms, C3 3.811 -> 3.582, C5 bf16
# 1.209 -> 1.110, its fp32 twin 1.423 -> 1.330, PACS 0.869 -> 0.808, MNIST neutral (its pairs are dual grids, which
# stay on the step's stream); 2 adds the decoder's first ConvTranspose2d (beside the latent launches): CelebA 1.928
# -> 1.887, C3 3.581 -> 3.532, C5 1.112 -> 1.097, PACS 0.805 -> 0.800.  1: without it; 0: one stream.
# CVHIP_WGRAD_LANES=2 (two side streams in rotation) measured neutral to slower (C5 1.112 -> 1.170 ms): default 1.
WGRAD_LANE = int(os.environ.get("CVHIP_WGRAD_LANE", "2"))  # (2: the decoder's first ConvTranspose2d too; 1: not it)
WGRAD_LANES = max(1, int(os.environ.get("CVHIP_WGRAD_LANES", "1")))  # side streams the weight gradients rotate over

# CVHIP_SPLIT_UPDATE=1: single-process steps with side-stream weight gradients reduce and update the decoder's
# parameters (cv_step_reduce of the decoder bucket, cv_adam_pack_step_part over the arena's decoder tail) on side
# lane 2 as soon as the step has read them (after the latent launches), beside the encoder backward; the encoder's
# reduction and Adam part (which advances the step counters) stay at the end.
SPLIT_UPDATE = os.environ.get("CVHIP_SPLIT_UPDATE", "0") == "1"


def disc_params(disc):
    """The factor discriminator of get_cleartcvae_trainer (trainer_utils.py:133-138) as a parameter list, or
    None when `disc` is not Linear(z, z) -> ReLU -> Linear(z, 1) -> Sigmoid."""
    import torch.nn as nn

    mods = list(disc) if isinstance(disc, nn.Sequential) else []
    if (len(mods) != 4 or not isinstance(mods[0], nn.Linear) or not isinstance(mods[1], nn.ReLU)
            or not isinstance(mods[2], nn.Linear) or not isinstance(mods[3], nn.Sigmoid)):
        return None
    l0, l2 = mods[0], mods[2]
    z = l0.in_features
    if l0.out_features != z or l2.in_features != z or l2.out_features != 1 or l0.bias is None or l2.bias is None:
        return None
    if z > 64 or z % 2:
        return None
    return [l0.weight, l0.bias, l2.weight, l2.bias]


def _dist_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


class _AdamState:
    """Flat Adam state bound to a torch.optim.Adam over exactly the params of `arena`."""

    def __init__(self, optimizer, arena: ParamArena):
        self.opt = optimizer
        self.arena = arena
        dev = arena.device
        self.m = torch.zeros(arena.numel, dtype=torch.float32, device=dev)
        self.v = torch.zeros(arena.numel, dtype=torch.float32, device=dev)
        steps = 0
        with torch.no_grad():
            for p in arena.params:
                st = optimizer.state.get(p, {})
                if "exp_avg" in st:
                    o, n = arena.offset[id(p)]
                    self.m[o:o + n].copy_(st["exp_avg"].reshape(-1))
                    self.v[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                    steps = int(float(st["step"]))
        self.host_steps = steps
        # [steps taken, arrival word, 64 group arrival words (cv_step_reduce_adam)]
        self.step = torch.zeros(2 + 64, dtype=torch.int64, device=dev)
        self.step[0] = steps
        self.hyper_host = None
        self.hyper = torch.zeros(8, dtype=torch.float32, device=dev)
        self.refresh_hyper()
        # bind optimizer.state to views of the flat state
        for p in arena.params:
            o, n = arena.offset[id(p)]
            optimizer.state[p] = {
                "step": torch.tensor(float(steps)),
                "exp_avg": self.m[o:o + n].view_as(p),
                "exp_avg_sq": self.v[o:o + n].view_as(p),
            }

    @staticmethod
    def supported(optimizer, params) -> bool:
        if type(optimizer) is not torch.optim.Adam or len(optimizer.param_groups) != 1:
            return False
        g = optimizer.param_groups[0]
        if g.get("amsgrad") or g.get("maximize") or g.get("differentiable") or g.get("decoupled_weight_decay"):
            return False
        if isinstance(g["lr"], torch.Tensor) or isinstance(g["betas"][0], torch.Tensor):
            return False
        ids = {id(p) for p in g["params"]}
        if ids != {id(p) for p in params} or not all(p.requires_grad for p in params):
            return False
        return True

    def refresh_hyper(self):
        g = self.opt.param_groups[0]
        h = (float(g["lr"]), float(g["betas"][0]), float(g["betas"][1]), float(g["eps"]), float(g["weight_decay"]))
        if h != self.hyper_host:
            self.hyper_host = h
            self.hyper.copy_(torch.tensor(list(h) + [0.0, 0.0, 0.0], dtype=torch.float32))

    def sync_host(self, n_new: int):
        self.host_steps += n_new
        for p in self.arena.params:
            st = self.opt.state[p]
            st["step"] = torch.tensor(float(self.host_steps))


class ClearStep:
    @classmethod
    def build(cls, trainer, mode: str):
        """Return a fused step for `trainer`, or None when its setup is outside the fused contract."""
        vae = trainer.model
        try:
            dev = next(vae.parameters()).device
        except StopIteration:
            return None
        if dev.type != "cuda" or trainer.transform is not None:
            return None
        try:
            arena = ensure_arena(vae)
        except (NotImplementedError, AssertionError):
            return None
        if not _AdamState.supported(trainer.optimizer, arena.params):
            return None
        if mode == "group":
            if getattr(vae, "mode", None) not in GROUP or vae._cv_spec.d > 64:
                return None
        elif trainer.sim_fn not in SIM:
            raise ValueError("unimplemented similarity measure.")
        if mode == "mim":
            from src.models.mi_estimator import CLUBSample, L1OutUB

            est = trainer.mi_estimator
            if type(est) not in (CLUBSample, L1OutUB):
                return None
            if not _AdamState.supported(trainer.mi_estimator_optimizer, est_params(est)):
                return None
        if mode == "tc":
            dp = disc_params(trainer.factor_cls)
            if dp is None or dp[0].shape[1] != 2 * vae._cv_spec.d:
                return None
            if next(trainer.factor_cls.parameters()).device != dev:
                return None
            if not _AdamState.supported(trainer.factor_optimizer, dp):
                return None
        return cls(trainer, mode)

    def __init__(self, trainer, mode: str):
        self.trainer = trainer
        self.mode = mode
        self.vae = trainer.model
        self.arena = ensure_arena(self.vae)
        self.spec = self.vae._cv_spec
        self.device = self.arena.device
        self.adam = _AdamState(trainer.optimizer, self.arena)
        hp = trainer.hyperparameter
        self.hp = dict(hp)
        self.sim = SIM[trainer.sim_fn] if mode != "group" else 0
        self.group_mode = GROUP[self.vae.mode] if mode == "group" else None
        self.anneal = torch.tensor([trainer.annealer.current_step], dtype=torch.int64, device=self.device)
        self.anneal_expected = trainer.annealer.current_step
        # the shared (device, seed) Philox counter: engine rebuilds and the module path (evaluate, fallback
        # steps) all advance one stream instead of replaying the same noise from 0
        self.seed, self.offset = rng.offset_tensor(self.device)
        self.world = _dist_world()
        # the data-parallel programs (segments + buckets); CVHIP_FORCE_DP=1 runs them in a world-1 process group too
        # (the one-GPU rehearsal of the RCCL paths: a SUM over one rank leaves the gradients as they are)
        self.dp = self.world > 1 or (os.environ.get("CVHIP_FORCE_DP", "0") == "1" and dist.is_available()
                                     and dist.is_initialized())
        self.capture_collectives = GRAPH_COLLECTIVES and self.dp
        # the VAE's Adam launch also packs the conv weights (ADAM_PACK); _packed_sig: the parameters' version
        # counters when the packed copies were last made current (None: unknown, pack before the next replay)
        ap = ADAM_PACK
        ap = (ap in (True, "1") or (ap not in (False, "0") and self.arena.numel >= ADAM_PACK_MIN))
        self.adam_pack = ap and not (FUSED_ADAM and not self.dp)
        self._packed_sig = None
        if self.world > 1:  # a noise stream per rank (the shards are different samples; equal noise would tie them)
            self.seed = (self.seed ^ (0x9E3779B97F4A7C15 * cvdist.rank())) & 0xFFFFFFFFFFFFFFFF
        self.gscale = torch.full((1,), 1.0 / self.world, dtype=torch.float32, device=self.device)
        self.graphs = {}  # n -> dict
        self.graphs_enabled = True
        self.steps_since_sync = 0
        if mode == "mim":
            self.est = trainer.mi_estimator
            self.est_arena = ParamArena(est_params(self.est), self.device)
            self.est_adam = _AdamState(trainer.mi_estimator_optimizer, self.est_arena)
            self.kind = MI_CLUBSAMPLE if type(self.est).__name__ == "CLUBSample" else MI_L1OUT
            self.learn = torch.zeros(5, dtype=torch.float32, device=self.device)
        if mode == "tc":  # the factor discriminator plays the estimator's part: its own arena + Adam
            self.est = trainer.factor_cls
            self.est_arena = ParamArena(disc_params(self.est), self.device)
            self.est_adam = _AdamState(trainer.factor_optimizer, self.est_arena)
            self.learn = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.two_nets = mode in ("mim", "tc")
        if self.dp:  # DDP construction semantics: every rank starts from rank 0's weights
            cvdist.broadcast_flat(self.arena.flat)
            if self.two_nets:
                cvdist.broadcast_flat(self.est_arena.flat)
            # captured collectives run on their own RCCL group built with the event cache off
            # (cvdist.captured_collectives_group: the abort a cached captured event causes cannot be reached,
            # whatever the default group's settings; a non-RCCL backend is refused here, before any capture)
            cgroup = cvdist.captured_collectives_group() if self.capture_collectives else None
            self.buckets = cvdist.GradBuckets(self.arena.grad, self.bucket_bounds(), group=cgroup, force=True)
            if self.two_nets:
                self.est_buckets = cvdist.GradBuckets(self.est_arena.grad, [(0, self.est_arena.numel)], group=cgroup,
                                                      force=True)
        # grads visible through p.grad (like the reference after loss.backward())
        for p in self.arena.params:
            p.grad = self.arena.gview(p)
        self._sig = self._signature()

    # ----------------------------------------------------------------------------- bookkeeping
    def _signature(self):
        t = self.trainer
        sig = (id(t.optimizer), getattr(t, "sim_fn", None),
               tuple(sorted((k, str(v)) for k, v in t.hyperparameter.items())),
               getattr(self.vae, "_cv_precision", "fp32"), getattr(self.vae, "mode", None))
        if self.mode == "mim":
            sig += (id(t.mi_estimator), id(t.mi_estimator_optimizer))
        if self.mode == "tc":
            sig += (id(t.factor_cls), id(t.factor_optimizer))
        return sig

    def compatible(self) -> bool:
        if self._signature() != self._sig or not self.arena.valid():
            return False
        if self.two_nets and not self.est_arena.valid():
            return False
        if self.anneal_expected != self.trainer.annealer.current_step:  # annealer changed by the caller
            self.anneal.fill_(self.trainer.annealer.current_step)
            self.anneal_expected = self.trainer.annealer.current_step
        return True

    # batch limit of the one-workgroup label segmentation (cv_group.hip GR_MAXN); larger group batches take
    # the module path instead of failing inside the step
    GROUP_MAXN = 4096

    def accepts(self, X) -> bool:
        sp = self.spec
        if self.mode == "group" and X.shape[0] > self.GROUP_MAXN:
            return False
        return (X.device.type == "cuda" and X.dim() == 4 and tuple(X.shape[1:]) == (sp.in_ch, sp.H, sp.W)
                and X.shape[0] >= 2)

    def resync_from_host(self):
        """After steps taken outside the engine (module path / torch Adam), adopt the host counters."""
        self.sync_host_state()
        st = self.trainer.optimizer.state.get(self.arena.params[0], {})
        if "step" in st:
            k = int(float(st["step"]))
            self.adam.host_steps = k
            self.adam.step.fill_(0)
            self.adam.step[0] = k
        for p in self.arena.params:
            p.grad = self.arena.gview(p)
        if self.two_nets:
            st = self.est_adam.opt.state.get(self.est_arena.params[0], {})
            if "step" in st:
                k = int(float(st["step"]))
                self.est_adam.host_steps = k
                self.est_adam.step.fill_(0)
                self.est_adam.step[0] = k

    def sync_host_state(self):
        if self.steps_since_sync:
            self.adam.sync_host(self.steps_since_sync)
            if self.two_nets:
                self.est_adam.sync_host((5 if self.mode == "mim" else 1) * self.steps_since_sync)
            self.steps_since_sync = 0

    # ----------------------------------------------------------------------------- programs
    def _programs(self, n: int):
        sp = self.spec
        ws = Workspace(sp, n, self.device, with_grad=True)
        X = torch.empty(n, sp.in_ch, sp.H, sp.W, dtype=torch.float32, device=self.device)
        lab = torch.zeros(n, dtype=torch.int64, device=self.device)
        A = self.arena
        hp = self.hp
        d = sp.d
        pg = A.gptr
        nslot = {"mim": 6, "tc": 2}.get(self.mode, 1)
        eps_buf = torch.zeros(nslot, n, 2 * d, dtype=torch.float32, device=self.device)  # test injection
        perm_buf = torch.zeros(n, dtype=torch.int64, device=self.device)
        grouped = self.mode == "group"
        if grouped:  # segmentation / group rows of cv_group_forward, and the B/m seed scale it writes
            gwork = torch.zeros(int(_lib.lib().cv_group_workspace_bytes(n, d)) // 4 + 4, dtype=torch.float32,
                                device=self.device)
            gscale_rec = torch.ones(1, dtype=torch.float32, device=self.device)

        # the contrastive branches (trainer.py:474-479): [mu_c, logvar_c] and [mu_s, logvar_s] of the heads, their
        # gradients into d(heads)
        hb = ws.heads.data_ptr()
        dh = ws.dheads.data_ptr()
        branches = None
        if not grouped:
            alpha = float(hp["alpha"])
            tau = float(hp["temperature"])
            branches = [cv_ntxent_branch(hb, hb + 4 * d, 4 * d, 0, dh, dh + 4 * d, 4 * d, None, alpha,
                                         ws.losses.data_ptr() + 12, ws.lse[0].data_ptr())]
        if self.mode == "clear":
            ps = bool(hp["ps"])
            branches.append(cv_ntxent_branch(hb + 8 * d, hb + 12 * d, 4 * d, int(ps), dh + 8 * d, dh + 12 * d, 4 * d,
                                             None, alpha if ps else -alpha, ws.losses.data_ptr() + 16,
                                             ws.lse[1].data_ptr()))
        br_arr = (cv_ntxent_branch * len(branches))(*branches) if branches is not None else None
        # NT-Xent beside the decoder (LATENT_SIDE): CLEAR / CLEAR-MIM steps captured as one graph
        side_nt = (LATENT_SIDE and br_arr is not None and self.mode in ("clear", "mim")
                   and (not self.dp or self.capture_collectives))
        aux_nt = (not side_nt and LATENT_AUX and br_arr is not None and self.mode in ("clear", "mim")
                  and len(sp.dec) >= 3)
        tau_c = ctypes.c_float(float(hp["temperature"])) if br_arr is not None else None
        aux_args = ([(br_arr, len(branches), lab, n, d, self.sim, tau_c, ph, 1) for ph in (0, 1)]
                    if aux_nt else None)
        chain_nt = aux_nt and LATENT_CHAIN and ws.fused_heads()
        # the phases in the decoder-input launches (LATENT_AUX_DL): phase 0 queued before the forward one, phase 1
        # before the backward one (each flushed right after its launch)
        dl_nt = (aux_nt and (LATENT_AUX_DL == 2 or (LATENT_AUX_DL == 1 and d > 8)) and not chain_nt
                 and not LATENT_AUX_OUT and ws.fused_decoder_input())
        hpf = lambda k, dflt: ctypes.c_float(float(hp.get(k, dflt)))
        aux_comb = ((ws.heads, ws.z, n, d, hpf("beta", 0), hpf("loc", 0), hpf("scale", 1), self.anneal, ws.dheads,
                     ws.losses) if chain_nt else None)
        chain = (cv_latent_chain(ws.heads.data_ptr(), ws.z.data_ptr(), ws.dz.data_ptr(), d, ws.rec.data_ptr(),
                                 ws.losses.data_ptr()) if chain_nt else None)

        def make_fwd(inject: bool):
            f = Program()
            # one launch refreshes the packed conv weights and zeroes the BN sums, the gradient arena and the
            # two split-K / accumulated latent buffers of the step (and d(heads) when the NT-Xent gradients
            # accumulate into it from the side stream)
            bufs = [(ws.stats, ws.stats.numel() * 8), (A.grad, A.numel * 4), (ws.heads, ws.heads.numel() * 4),
                    (ws.dz, ws.dz.numel() * 4)]
            if side_nt or aux_nt:
                bufs.append((ws.dheads, ws.dheads.numel() * 4))
            pack_program(sp, f, "all", zero=bufs)
            rp = None if grouped else (eps_buf[0] if inject else None, self.seed, self.offset)
            drew = ws.encoder_program(f, X, True, zero_heads=False, reparam=rp)
            if side_nt:  # row log-sum-exps + gradients of both branches on the side stream (joined in `lat`)
                f.add_fork("cv_ntxent", br_arr, len(branches), lab, n, d, self.sim, ctypes.c_float(tau), 2, 1)
                f.keep.append(br_arr)
                f.join_at_end = False
            if grouped:
                hb = ws.heads.data_ptr()
                f.add("cv_group_forward", self.group_mode, hb, hb + 4 * d, 4 * d, lab, n, d, gwork, gscale_rec,
                      hb + 8 * d, hb + 12 * d, 4 * d, eps_buf[0] if inject else None, 2 * d, ctypes.c_uint64(self.seed),
                      None if inject else self.offset, ws.z)
                ws.decoder_program(f, ws.z, True, "loss", X, rec_scale=gscale_rec)
                f.keep += [gwork, gscale_rec]
            else:
                ws.decoder_program(f, ws.z, True, "loss", X, reparam=None if drew else rp,
                                   aux=None if dl_nt else aux_args, aux_combine=aux_comb,
                                   aux_at=(0, len(sp.dec) - 1) if LATENT_AUX_OUT else None,
                                   aux_in=aux_args[0] if dl_nt else None)
                if aux_nt:
                    f.keep.append(br_arr)
            # (the running statistics are folded at the end of the backward by cv_step_reduce)
            return f

        fwd, fwd_inj = make_fwd(False), make_fwd(True)
        # the replayed step's graph starts after the pack + zero launch: step() issues that launch eagerly with the
        # batch copy into X / lab folded in (cv_pack_conv_weights_zero_copy: one launch instead of two)
        pack_call = fwd.calls[0]
        assert pack_call[0] == "cv_pack_conv_weights_zero", pack_call[0]
        fwd_g = Program()
        fwd_g.calls = fwd.calls[1:]
        fwd_g.keep = fwd.keep
        # decoder backward (bucket 1 of the gradient arena).  Weight gradients are deferred: their split-K
        # partial tiles, the BN affine gradients and the running statistics are reduced by one
        # cv_step_reduce launch at the end of the backward (data parallel: one per gradient bucket, before
        # the bucket's all-reduce)
        dp = self.dp
        adam_pack = self.adam_pack
        dec_defer, enc_defer = DeferGroup(), DeferGroup()
        ws.wgrad_side = WGRAD_LANE >= 1
        ws.wgrad_side_first = WGRAD_LANE >= 2
        ws.wgrad_lanes = WGRAD_LANES
        ws._wside_next = 0
        dec = Program()
        det_dz = DET_DZ and (side_nt or aux_nt) and not chain_nt and ws.fused_decoder_input()
        ws.decoder_backward_program(dec, pg, ws.dz, zero_dz=False, defer=dec_defer if dp else enc_defer,
                                    aux_in=aux_args[1] if dl_nt else None, dz_later=det_dz)
        if dl_nt:
            dec.keep.append(br_arr)
        if dp:
            if ws.wgrad_side:
                dec.add_join(ws.side_lanes())
            ws.step_reduce_program(dec, dec_defer, pg, "dec", running=False)

        # latent terms -> d(heads)
        lat = Program()
        if grouped:
            lat.add("cv_group_backward", self.group_mode, ws.heads, ws.z, ws.dz, gwork, n, d,
                    ctypes.c_float(float(hp["beta"])), ctypes.c_float(float(hp.get("loc", 0))),
                    ctypes.c_float(float(hp.get("scale", 1))), self.anneal, ws.rec, ws.dheads, ws.losses)
            lat_inj = lat
            lat.keep.append(gwork)
        elif chain_nt:  # (the combine's two parts ride in the rows-phase grid and in the heads backward)
            lat_inj = Program()
        elif side_nt or aux_nt:
            # (side stream: join it first) the KL + decoder-chain seed added onto the NT-Xent gradients
            if side_nt:
                lat.add_join()
            if det_dz:  # (dz = d(h) W here, in fixed order, written to ws.dz for any later reader)
                lat.add("cv_latent_combine_dz", ws.heads, ws.z, ws.gah, sp.dec_lin.weight, ws.decoder_input_geometry(),
                        ctypes.c_float(float(hp["beta"])), ctypes.c_float(float(hp.get("loc", 0))),
                        ctypes.c_float(float(hp.get("scale", 1))), self.anneal, ws.rec, ws.dheads, ws.losses, ws.dz,
                        1, ws.comb_dz_work)
            else:
                lat.add("cv_latent_combine_acc", ws.heads, ws.z, ws.dz, n, d, ctypes.c_float(float(hp["beta"])),
                        ctypes.c_float(float(hp.get("loc", 0))), ctypes.c_float(float(hp.get("scale", 1))),
                        self.anneal, ws.rec, ws.dheads, ws.losses, ws.comb_work)
            lat_inj = Program()
            lat_inj.extend(lat)
        if branches is not None and not side_nt and not aux_nt:
            arr = br_arr
            # KL + decoder chain into d(heads) with the contrastive terms accumulated on top
            lat.add("cv_latent_step", ws.heads, ws.z, ws.dz, n, d, ctypes.c_float(float(hp["beta"])),
                    ctypes.c_float(float(hp.get("loc", 0))), ctypes.c_float(float(hp.get("scale", 1))), self.anneal,
                    ws.rec, ws.dheads, ws.losses, arr, len(branches), lab, self.sim, ctypes.c_float(tau))
            lat.keep.append(arr)
            lat_inj = Program()
            lat_inj.extend(lat)
        if self.mode == "mim":
            mlp = mlp_struct(self.est)
            zp = ws.z.data_ptr()
            for prog, pin in ((lat, None), (lat_inj, perm_buf)):
                prog.add("cv_mi_forward", self.kind, mlp, zp, 2 * d, zp + 4 * d, 2 * d, n, pin,
                         ctypes.c_uint64(self.seed), self.offset, ws.mi_work, ws.losses.data_ptr() + 20)
                prog.add("cv_mi_backward", self.kind, mlp, zp, 2 * d, zp + 4 * d, 2 * d, n, ws.mi_work, None,
                         ctypes.c_float(float(hp["lambda"])), None, None, 0, 1, None, ws.heads, ws.z, ws.dheads, d)
        if self.mode == "tc":  # relu(log(D/(1-D))).mean() and lambda * its gradient into d(heads)
            disc = self._disc_struct()
            tc_work = torch.zeros(int(_lib.lib().cv_tc_workspace_bytes(2 * d)) // 4 + 4, dtype=torch.float32,
                                  device=self.device)
            for prog in (lat, lat_inj):
                prog.add("cv_tc_forward", disc, ws.z, n, ctypes.c_float(float(hp["lambda"])), ws.heads, ws.dheads,
                         d, tc_work, ws.losses.data_ptr() + 20)
        enc = Program()
        enc2 = None
        if dp:
            # the encoder gradients in two buckets at layer `k`: the heads and the deep convs (layers >= k, the
            # bulk of the encoder's parameters) are reduced and all-reduced as soon as their weight gradients
            # are in, while the shallow layers' backward (the big-grid GEMMs) still runs; the shallow bucket
            # follows with every layer's running statistics
            k = self._enc_split()
            nl = len(sp.enc)
            enc_defer2 = DeferGroup()
            ws.encoder_backward_program(enc, pg, ws.dheads, x=X, defer=enc_defer, layers=range(nl - 1, k - 1, -1),
                                        chain=chain)
            if ws.wgrad_side:
                enc.add_join(ws.side_lanes())
            ws.step_reduce_program(enc, enc_defer, pg, ws.bn_enc[k:], running=False)
            enc2 = Program()
            ws.encoder_backward_program(enc2, pg, ws.dheads, x=X, defer=enc_defer2, heads=False,
                                        layers=range(k - 1, -1, -1))
            if ws.wgrad_side:
                enc2.add_join(ws.side_lanes())
            ws.step_reduce_program(enc2, enc_defer2, pg, ws.bn_enc[:k], running=False)
            ws.running_program(enc2, "all")
        else:
            ws.encoder_backward_program(enc, pg, ws.dheads, x=X, defer=enc_defer, chain=chain)
        upd = Program()
        items = sp.pack_items["enc"] + sp.pack_items["dec"]
        pack_arr = struct_array(cv_conv_pack, items)
        adam_name = "cv_adam_pack_step" if adam_pack else "cv_adam_step"
        adam_tail = (pack_arr, len(items)) if adam_pack else ()
        if dp:
            upd.add(adam_name, A.flat, A.grad, self.adam.m, self.adam.v, A.numel, self.adam.hyper,
                    self.adam.step, self.gscale, self.anneal, *adam_tail)
        elif not FUSED_ADAM:
            if ws.wgrad_side:
                enc.add_join(ws.side_lanes())
            ws.step_reduce_program(enc, enc_defer, pg, "all", running=True)
            upd.add(adam_name, A.flat, A.grad, self.adam.m, self.adam.v, A.numel, self.adam.hyper,
                    self.adam.step, None, self.anneal, *adam_tail)
        else:  # single process: the optimizer step rides in the end-of-backward reduction launch
            if ws.wgrad_side:
                enc.add_join(ws.side_lanes())
            ws.step_reduce_program(enc, enc_defer, pg, "all", running=True,
                                   adam=(A.flat, A.grad, self.adam.m, self.adam.v, A.numel, self.adam.hyper,
                                         self.adam.step, self.anneal))
        if adam_pack:
            upd.keep.append(pack_arr)
        # the split update (SPLIT_UPDATE): the decoder bucket's reduction and Adam on side lane 2 once the step has
        # read the decoder's parameters (after `lat`), beside the encoder backward; `dec_p` / `enc_p` / `upd_p` keep
        # the one-update form for steps with a before_update hook (which reads the pre-update decoder BatchNorm)
        dec_p, enc_p, upd_p = dec, enc, upd
        split = self._split_update_plan(ws, sp, A) if (SPLIT_UPDATE and adam_pack and ws.wgrad_side and not dp
                                                       and not FUSED_ADAM) else None
        if split is not None:
            dec_off, dec_items, enc_items = split
            dec_defer_s, enc_defer_s = DeferGroup(), DeferGroup()
            ws._wside_next = 0
            dec = Program()
            ws.decoder_backward_program(dec, pg, ws.dz, zero_dz=False, defer=dec_defer_s,
                                        aux_in=aux_args[1] if dl_nt else None, dz_later=det_dz)
            if dl_nt:
                dec.keep.append(br_arr)
            enc = Program()
            enc.add_join([1])  # (the decoder's weight gradients, issued on side lane 1 by the `dec` calls)
            side = Program()
            ws.step_reduce_program(side, dec_defer_s, pg, "dec", running=True)
            darr = struct_array(cv_conv_pack, dec_items)
            f4 = 4 * dec_off
            side.add("cv_adam_pack_step_part", A.flat.data_ptr() + f4, A.grad.data_ptr() + f4,
                     self.adam.m.data_ptr() + f4, self.adam.v.data_ptr() + f4, A.numel - dec_off, self.adam.hyper,
                     self.adam.step, None, self.anneal, darr, len(dec_items), 0)
            side.keep.append(darr)
            enc.extend(side, lane=2)
            ws.encoder_backward_program(enc, pg, ws.dheads, x=X, defer=enc_defer_s, chain=chain)
            enc.add_join(ws.side_lanes() + [2])
            ws.step_reduce_program(enc, enc_defer_s, pg, ws.bn_enc, running=True)
            upd = Program()
            earr = struct_array(cv_conv_pack, enc_items)
            upd.add("cv_adam_pack_step_part", A.flat, A.grad, self.adam.m, self.adam.v, dec_off, self.adam.hyper,
                    self.adam.step, None, self.anneal, earr, len(enc_items), 1)
            upd.keep.append(earr)
        learn = learn_inj = None
        if self.mode == "mim":
            E = self.est_arena
            mlp = mlp_struct(self.est)
            G = cv_mlp_grad(*[E.gptr(p) for p in est_params(self.est)])
            zp = ws.z.data_ptr()

            # The 5 estimator updates (trainer.py:873-888) each run a train-mode forward of the same batch through
            # the same (post-Adam) VAE: the encoder, its batch statistics and the heads are identical in all five,
            # so they are computed once; each update re-runs the reparameterisation (fresh noise), the decoder
            # (its statistics follow z) and the running-statistics update of every layer (the encoder's five
            # momentum updates with its one set of batch statistics, as in five forwards)
            # (the statistics of the first estimator forward are zeroed by the pack launch before it)
            stats_zero = [(ws.stats, ws.stats.numel() * 8)]

            def learn_forward(prog, j, inject):
                rp = (eps_buf[1 + j] if inject else None, self.seed, self.offset)
                if j == 0:
                    if ws.encoder_program(prog, X, True, reparam=rp):
                        return None  # (z drawn by the heads launch)
                else:
                    prog.add("cv_zero_many", ptr_array([ws.dec_stats.data_ptr(), ws.dec_tickets.data_ptr()]),
                             (ctypes.c_size_t * 2)(ws.dec_stats.numel() * 8, ws.dec_tickets.numel() * 8), 2)
                return rp

            def make_learn(inject: bool):
                lp = Program()
                # the VAE Adam step just moved the weights (ADAM_PACK: and packed them)
                pack_program(sp, lp, None if adam_pack else "all", zero=stats_zero)
                for j in range(5):
                    ws.decoder_program(lp, ws.z, True, "none", reparam=learn_forward(lp, j, inject))
                    ws.running_program(lp, "all")
                    lp.add("cv_mi_learning_step", mlp, zp, 2 * d, zp + 4 * d, 2 * d, n, ws.mi_work,
                           self.learn.data_ptr() + 4 * j, G, E.flat, E.grad, self.est_adam.m, self.est_adam.v,
                           E.numel, self.est_adam.hyper, self.est_adam.step)
                return lp

            # MIM_BRANCHES > 0: the five decoder forwards are independent of each other and of the estimator (update j
            # reads only z_j, and its decoder pass only feeds the running statistics), so once the encoder pass has
            # run and the five z_j are drawn in order on the step's stream (the noise of the sequential form, draw by
            # draw), update j's decoder forward runs on side lane 1 + j % MIM_BRANCHES of the graph with its own
            # activations, statistics and in-launch split-K workspace, while the step's stream runs the five
            # estimator learning steps (each needs only z_j and the previous step's estimator); after the join the
            # running statistics take their five momentum updates in order, as five forwards would have.
            nbr = MIM_BRANCHES
            if nbr > 0:
                bws = [ws] + [Workspace(sp, n, self.device, with_grad=False, encoder=False) for _ in range(4)]
                nb_fix = int(_lib.lib().cv_gemm_workspace_bytes())
                fixws = [torch.zeros((nb_fix + 15) // 16 * 4, dtype=torch.float32, device=self.device)
                         for _ in range(nbr)]
                dflt_fix = _lib.gemm_workspace(self.device)
                set_fix = lambda buf: _lib.call("cv_set_gemm_workspace", buf.data_ptr(), buf.numel() * 4)  # noqa: E731

            def make_learn_branched(inject: bool):
                lp = Program()
                # the VAE Adam step just moved the weights; the same launch zeroes every update's statistics
                pack_program(sp, lp, None if adam_pack else "all", zero=[(w.stats, w.stats.numel() * 8) for w in bws])
                rp = (eps_buf[1] if inject else None, self.seed, self.offset)
                zs = [ws.z] + [w.z for w in bws[1:]]
                if not ws.encoder_program(lp, X, True, reparam=rp):  # (z_0 drawn by the heads launch, or here)
                    lp.add("cv_reparam_forward", ws.heads, n, d, rp[0], ctypes.c_uint64(self.seed), self.offset,
                           zs[0], None)
                for j in range(1, 5):
                    lp.add("cv_reparam_forward", ws.heads, n, d, eps_buf[1 + j] if inject else None,
                           ctypes.c_uint64(self.seed), None if inject else self.offset, zs[j], None)
                # per lane: its decoder forwards (lanes 1..nbr) or the five learning steps (lane nbr + 1); every lane
                # forks once, after the draws.  The calls are enqueued round-robin over the lanes, so the graph's nodes
                # are created (and submitted at each launch) interleaved and no lane's first kernel waits behind
                # another lane's whole chain (a multi-queue graph launch submits its nodes at ~25 us each, measured)
                lanes = {k: [] for k in range(1, nbr + 2)}
                for j in range(5):
                    br = Program()
                    bws[j].decoder_program(br, zs[j], True, "none")
                    lp.keep += br.keep
                    lanes[1 + j % nbr] += br.calls
                for j in range(5):
                    zj = zs[j].data_ptr()
                    lp.add("cv_mi_learning_step", mlp, zj, 2 * d, zj + 4 * d, 2 * d, n, ws.mi_work,
                           self.learn.data_ptr() + 4 * j, G, E.flat, E.grad, self.est_adam.m, self.est_adam.v,
                           E.numel, self.est_adam.hyper, self.est_adam.step)
                    nm, fn, a, _ = lp.calls.pop()
                    lanes[nbr + 1].append((nm, fn, a, nbr + 1))
                queues = {k: [(c[0], c[1], c[2], k) for c in v] for k, v in lanes.items()}
                while any(queues.values()):
                    for k, q in queues.items():
                        if q:
                            if k <= nbr:  # (each decoder lane's launches take that lane's split-K workspace)
                                lp.add_host("gemm_workspace", set_fix, fixws[k - 1])
                            lp.calls.append(q.pop(0))
                lp.add_host("gemm_workspace", set_fix, dflt_fix)
                lp.add_join()
                ws.running_sets_program(lp, [ws.bn_enc + [bws[j].bn_1d] + bws[j].bn_dec for j in range(5)])
                lp.keep += fixws + bws[1:]
                return lp

            def make_learn_dp(inject: bool):
                # per estimator update: (forward + learning-loss gradients, Adam) with the estimator
                # gradient all-reduced in between
                out = []
                for j in range(5):
                    gp = Program()
                    if j == 0:
                        pack_program(sp, gp, None if adam_pack else "all", zero=stats_zero)
                    ws.decoder_program(gp, ws.z, True, "none", reparam=learn_forward(gp, j, inject))
                    ws.running_program(gp, "all")
                    gp.add("cv_mi_learning_step", mlp, zp, 2 * d, zp + 4 * d, 2 * d, n, ws.mi_work,
                           self.learn.data_ptr() + 4 * j, G, None, None, None, None, 0, None, None)
                    ap = Program()
                    ap.add("cv_adam_step", E.flat, E.grad, self.est_adam.m, self.est_adam.v, E.numel,
                           self.est_adam.hyper, self.est_adam.step, self.gscale, None)
                    out.append((gp, ap))
                return out

            if self.dp:
                learn, learn_inj = make_learn_dp(False), make_learn_dp(True)
            elif nbr > 0:
                learn, learn_inj = make_learn_branched(False), make_learn_branched(True)
            else:
                learn, learn_inj = make_learn(False), make_learn(True)
        if self.mode == "tc":
            E = self.est_arena
            disc = self._disc_struct()
            G = cv_tc_grad(*[E.gptr(p) for p in E.params])

            def make_tc(inject: bool):
                # trainer.py:680-699: a second train-mode forward (fresh noise) on the updated VAE, then the
                # discriminator's BCE gradients and its Adam step (data parallel: all-reduce in between)
                gp = Program()
                # the VAE Adam step just moved the weights; the same launch zeroes the forward's statistics
                pack_program(sp, gp, None if adam_pack else "all", zero=[(ws.stats, ws.stats.numel() * 8)])
                rp = (eps_buf[1] if inject else None, self.seed, self.offset)
                drew = ws.encoder_program(gp, X, True, reparam=rp)
                ws.decoder_program(gp, ws.z, True, "none", reparam=None if drew else rp)
                ws.running_program(gp, "all")
                gp.add("cv_tc_learning_step", disc, ws.z, n, tc_work, self.learn, G)
                ap = Program()
                ap.add("cv_adam_step", E.flat, E.grad, self.est_adam.m, self.est_adam.v, E.numel,
                       self.est_adam.hyper, self.est_adam.step, self.gscale if self.dp else None, None)
                if self.dp:
                    return [(gp, ap)]
                gp.extend(ap)
                return gp

            learn, learn_inj = make_tc(False), make_tc(True)
        return dict(ws=ws, X=X, lab=lab, fwd=fwd, dec=dec, lat=lat, enc=enc, enc2=enc2, upd=upd, learn=learn,
                    dec_p=dec_p, enc_p=enc_p, upd_p=upd_p,
                    fwd_inj=fwd_inj, lat_inj=lat_inj, learn_inj=learn_inj, eps_buf=eps_buf, perm_buf=perm_buf,
                    fwd_g=fwd_g, pack_call=pack_call)

    def _split_update_plan(self, ws, sp, A):
        """(decoder arena offset, decoder pack items, encoder pack items) when the decoder's parameters are the
        arena's tail and every pack item lies on its side of that offset (the split update's two Adam parts), else
        None."""
        base = A.flat.data_ptr()
        dec_params = [p for k, p in self.vae.named_parameters() if k.startswith("decoder.")]
        if not dec_params:
            return None
        dec_ids = {id(p) for p in dec_params}
        dec_off = min((p.data_ptr() - base) // 4 for p in dec_params)
        for p in A.params:
            if (((p.data_ptr() - base) // 4) >= dec_off) != (id(p) in dec_ids):
                return None
        ei, di = sp.pack_items["enc"], sp.pack_items["dec"]
        if not ei or not di:
            return None
        if any(it.src - base < 4 * dec_off for it in di) or any(it.src - base >= 4 * dec_off for it in ei):
            return None
        return dec_off, di, ei

    def _disc_struct(self) -> cv_tc_disc:
        l0w, l0b, l2w, l2b = self.est_arena.params
        return cv_tc_disc(l0w.data_ptr(), l0b.data_ptr(), l2w.data_ptr(), l2b.data_ptr(), l0w.shape[1])

    def _bucket_split(self):
        """Offset of the first decoder parameter in the arena (decoder grads = [split, numel))."""
        sp = self.spec
        return self.arena.offset[id(sp.dec_lin.weight)][0]

    def _enc_split(self) -> int:
        """First conv layer of the deep encoder bucket: the deepest layers that, with the heads, hold >= 80 % of
        the encoder's parameters (VAE64: conv4, conv5 + heads, 2.9 M of 3.1 M; VAE: conv3 + heads, 140 k of
        158 k).  The deep bucket's all-reduce runs while the shallow layers' backward (the big-grid GEMMs)
        still runs; the shallow bucket (VAE64 0.66 MB, VAE 75 KB) is the exposed part."""
        sp = self.spec
        size = [c.mod.weight.numel() + c.mod.bias.numel() + 2 * c.bn.num_features for c in sp.enc]
        heads = sum(h.weight.numel() + h.bias.numel() for h in sp.heads)
        total = sum(size) + heads
        k, acc = len(sp.enc), heads
        while k > 1 and acc < 0.8 * total:
            k -= 1
            acc += size[k]
        return k if k < len(sp.enc) else len(sp.enc) - 1

    def bucket_bounds(self):
        """Gradient buckets in launch order (element ranges of the arena): decoder, deep encoder (the heads
        and layers >= _enc_split()), shallow encoder."""
        split = self._bucket_split()
        k = self._enc_split()
        mid = self.arena.offset[id(self.spec.enc[k].mod.weight)][0]
        return [(split, self.arena.numel), (mid, split), (0, mid)]

    def _segments(self, G, inject=False, graph=False):
        """The step as ('prog', [Program...]) segments and ('ar', bucket) / ('ar_est',) / ('wait',)
        points (single GPU: one segment).  graph=True: the programs a step graph is captured from (the step's
        first launch, pack + zero, is issued before the graph with the batch copy: _pack_and_load)."""
        fwd = G["fwd_inj" if inject else ("fwd_g" if graph else "fwd")]
        lat = G["lat_inj" if inject else "lat"]
        learn = G["learn_inj" if inject else "learn"]
        if not self.dp:
            progs = [fwd, G["dec"], lat, G["enc"], G["upd"]] + ([learn] if learn is not None else [])
            return [("prog", progs)]
        seg = [("prog", [fwd, G["dec"]]), ("ar", 0), ("prog", [lat, G["enc"]]), ("ar", 1), ("prog", [G["enc2"]]),
               ("ar", 2), ("wait",), ("prog", [G["upd"]])]
        if learn is not None:
            for gp, ap in learn:
                seg += [("prog", [gp]), ("ar_est",), ("wait_est",), ("prog", [ap])]
        return seg

    def _run_segments(self, segs, graphs=None, upd=None, before_update=None):
        s = _lib.stream_handle()
        gi = 0
        for item in segs:
            kind = item[0]
            if kind == "prog":
                if graphs is None:
                    for P in item[1]:
                        if before_update is not None and P is upd:
                            before_update()
                        P.run(s)
                else:
                    graphs[gi].replay()
                    gi += 1
            elif kind == "ar":
                self.buckets.launch(item[1])
            elif kind == "wait":
                self._probe_wait(self.buckets)
            elif kind == "ar_est":
                self.est_buckets.launch(0)
            elif kind == "wait_est":
                self._probe_wait(self.est_buckets)

    # comm_probe: None, or a list receiving (kind, start, end) HIP events around every wait for the gradient
    # all-reduce on the step's stream: the exposed (not overlapped) collective time (bench.py)
    comm_probe = None

    def _probe_wait(self, buckets):
        if self.comm_probe is None:
            buckets.wait()
            return
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        buckets.wait()
        e1.record()
        self.comm_probe.append(("vae" if buckets is self.buckets else "est", e0, e1))

    def _run_eager(self, G, inject=False, before_update=None):
        if before_update is not None and G.get("dec_p") is not None and G["dec_p"] is not G["dec"]:
            # (the one-update programs: the hook reads the step's state before any parameter moves)
            H = dict(G, dec=G["dec_p"], enc=G["enc_p"], upd=G["upd_p"])
            self._run_segments(self._segments(H, inject), upd=H["upd"], before_update=before_update)
            return
        self._run_segments(self._segments(G, inject), upd=G["upd"], before_update=before_update)

    def _take_injections(self, G) -> bool:
        """Consume queued test noise (cvhip.rng): eps_c, eps_s for the main forward and, in CLEAR-MIM,
        5 more pairs for the estimator forwards plus one CLUB-S permutation; in CLEAR-TC one more pair for
        the discriminator step's forward."""
        need = 2 * {"mim": 6, "tc": 2}.get(self.mode, 1)
        if rng.pending_noise() < need:
            return False
        d = self.spec.d
        for slot in range(need // 2):
            ec, es = rng.next_noise(), rng.next_noise()
            G["eps_buf"][slot, :, :d].copy_(ec)
            G["eps_buf"][slot, :, d:].copy_(es)
        if self.mode == "mim":
            pm = rng.next_perm()
            if pm is None:
                raise RuntimeError("CLEAR-MIM injection needs a permutation (cvhip.rng.inject_perm)")
            G["perm_buf"].copy_(pm)
        return True

    def _capture(self, G):
        """One executable HIP graph per program segment (_lib.StepGraph: launched directly, without
        PyTorch's per-replay RNG bookkeeping); with capture_collectives, one graph for the whole data-parallel step,
        its all-reduces captured between the segments (the first, eager step has created the communicators)."""
        if self.capture_collectives:
            def record_all(s, segs=self._segments(G, False, graph=PACK_COPY)):
                for item in segs:
                    kind = item[0]
                    if kind == "prog":
                        for P in item[1]:
                            P.run(s)
                    elif kind == "ar":
                        self.buckets.launch(item[1])
                    elif kind == "wait":
                        self.buckets.wait()
                    elif kind == "ar_est":
                        self.est_buckets.launch(0)
                    elif kind == "wait_est":
                        self.est_buckets.wait()

            G["graphs"] = [_lib.StepGraph(record_all)]
            G["one_graph"] = True
            return
        graphs = []
        for item in self._segments(G, False, graph=PACK_COPY):
            if item[0] != "prog":
                continue

            def record(s, progs=item[1]):
                for P in progs:
                    P.run(s)

            graphs.append(_lib.StepGraph(record))
        G["graphs"] = graphs

    # ----------------------------------------------------------------------------- one step
    def _load_batch(self, G, X, label):
        """Copy the batch into the graph's static input buffers (one launch when no conversion is needed)."""
        lab = label.reshape(-1)
        if (X.dtype == torch.float32 and X.is_contiguous() and X.device == G["X"].device and lab.dtype == torch.int64
                and lab.is_contiguous() and lab.device == G["lab"].device):
            dst = ptr_array([G["X"].data_ptr(), G["lab"].data_ptr()])
            src = ptr_array([X.data_ptr(), lab.data_ptr()])
            nb = (ctypes.c_size_t * 2)(G["X"].numel() * 4, G["lab"].numel() * 8)
            _lib.call("cv_copy_many", dst, src, nb, 2, _lib.stream_handle())
        else:
            G["X"].copy_(X, non_blocking=True)
            G["lab"].copy_(lab, non_blocking=True)

    PACK_COPY_MAX = int(os.environ.get("CVHIP_PACK_COPY_MAX", str(4 << 20)))  # bytes

    def _pack_and_load(self, G, X, label):
        """The replayed step's first launch: the weight packing and step zeroing of the `fwd` program with the
        batch copy into the graph's static inputs folded in (one launch), or the copy by torch and the packing on
        its own when the batch needs a conversion."""
        lab = label.reshape(-1)
        name, fn, args, _ = G["pack_call"]
        if self.adam_pack:
            if self._packed_sig != self._param_sig():  # (parameters changed outside the engine: repack first)
                _lib.call("cv_pack_conv_weights", args[0], args[1], _lib.stream_handle())
            args = (None, 0) + tuple(args[2:])  # (the packed copies are current: zero / copy only)
        nbx, nbl = G["X"].numel() * 4, G["lab"].numel() * 8
        # (folded in for small batches only: the pack launch's workgroups hold a 35 KB LDS tile each, so a large copy
        # — VAE64 bs = 256: 12.6 MB — runs slower inside it than as its own launch: CelebA +3 us, MNIST -3 us, measured)
        if (X.dtype == torch.float32 and X.is_contiguous() and X.device == G["X"].device and lab.dtype == torch.int64
                and lab.is_contiguous() and lab.device == G["lab"].device and X.numel() * 4 == nbx
                and lab.numel() * 8 == nbl and nbx % 16 == 0 and nbl % 16 == 0
                and (X.data_ptr() | lab.data_ptr()) % 16 == 0 and nbx + nbl <= self.PACK_COPY_MAX):
            dst = ptr_array([G["X"].data_ptr(), G["lab"].data_ptr()])
            src = ptr_array([X.data_ptr(), lab.data_ptr()])
            nb = (ctypes.c_size_t * 2)(nbx, nbl)
            _lib.call("cv_pack_conv_weights_zero_copy", *args, dst, src, nb, 2, _lib.stream_handle())
            return
        self._load_batch(G, X, label)
        rc = fn(*args, _lib.stream_handle())
        if rc != 0:
            _lib.check(rc, name)

    def _param_sig(self):
        # (the parameters' own counters — load_state_dict, torch optimizers — and the arena's: writes into the flat
        # buffer or its views; only `.data` aliases escape both)
        sig = (self.arena.flat._version,) + tuple(p._version for p in self.arena.params)
        if self.two_nets:
            sig += (self.est_arena.flat._version,) + tuple(p._version for p in self.est_arena.params)
        return sig

    def invalidate_packed(self):
        """Repack the conv weights before the next replayed step (after parameters were changed through `.data`,
        which the version counters ADAM_PACK watches do not see)."""
        self._packed_sig = None

    def step(self, X, label, before_update=None):
        """One training step on the batch (X, label).  before_update: an optional callable run (on the host, in
        stream order: the step's kernels before it are enqueued, none after) once the gradients are complete —
        all-reduced under DP — and before the Adam launch; such a step runs eagerly, not from the graph (used by
        the tests to read the step's activations with the pre-update parameters)."""
        n = X.shape[0]
        if before_update is not None and FUSED_ADAM and not self.dp:
            # (Adam rides in the reduction launch of the `enc` program: there is no point between the complete
            # gradients and the update at which the hook could run)
            raise RuntimeError("before_update is not supported with CVHIP_FUSED_ADAM=1")
        G = self.graphs.get(n)
        if G is None:
            G = self._programs(n)
            G["count"] = 0
            self.graphs[n] = G
        self.adam.refresh_hyper()
        if self.two_nets:
            self.est_adam.refresh_hyper()
        inject = self._take_injections(G)
        use_graph = G["count"] >= 1 and not inject and self.graphs_enabled and before_update is None
        if use_graph and "graphs" not in G:
            self._capture(G)
        if use_graph and PACK_COPY:
            self._pack_and_load(G, X, label)
        else:
            self._load_batch(G, X, label)
        if use_graph and G.get("one_graph"):
            G["graphs"][0].replay()  # (the whole step, collectives included: one launch)
        elif use_graph:
            self._run_segments(self._segments(G, False), G["graphs"])
        else:
            self._run_eager(G, inject, before_update)
        G["count"] += 1
        if self.adam_pack:  # (the step's Adam launch packed the weights it updated)
            self._packed_sig = self._param_sig()
        self.steps_since_sync += 1
        self.anneal_expected += 1
        ws = G["ws"]
        if self.two_nets:  # (CLEAR-MIM: the 5 learning losses; CLEAR-TC: the discriminator's BCE)
            return ws.losses, self.learn.clone()
        return ws.losses

    def last_workspace(self, n):
        return self.graphs[n]["ws"]
