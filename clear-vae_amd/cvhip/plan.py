"""Layer plan of a CLEAR-VAE model on the HIP kernels.

``VaeSpec`` reads the topology of a ``VAE`` / ``VAE64`` module (code/src/models/vae.py:7-156 of the
reference): the conv encoder, the four latent heads, the decoder Linear -> BatchNorm1d -> ReLU ->
Unflatten, the transposed-conv decoder and the BatchNorm + Sigmoid output.

``ParamArena`` moves every parameter of a module into one flat fp32 buffer (params become views), so
the whole model's gradient, Adam state and data-parallel all-reduce are single contiguous buffers.

``Workspace`` holds the per-batch-size device buffers (NHWC activations, gradients, fp64 BatchNorm
statistics) and ``Program`` a pre-built list of C-ABI calls over them; the fused trainer captures a
program into a HIP graph, the autograd path runs it eagerly.
"""

from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import torch
import torch.nn as nn

from . import _lib
from ._lib import (
    STAT_BWD,
    STAT_FWD,
    STAT_NONE,
    XF_BNBWD,
    XF_BNRELU,
    XF_NONE,
    cv_bn,
    cv_conv,
    cv_conv_pack,
    cv_epilogue,
    cv_linear,
    cv_operand,
    cv_wgrad_defer,
)

# ----------------------------------------------------------------------------- topology


@dataclass
class ConvSpec:
    mod: nn.Module  # nn.Conv2d or nn.ConvTranspose2d
    bn: nn.Module  # BatchNorm2d after it
    relu: bool  # ReLU after the BN (False for the decoder output: Sigmoid)
    transposed: bool
    c_in: int
    h_in: int
    w_in: int
    c_out: int
    h_out: int
    w_out: int
    # GEMM-native weight copies (cv_pack_conv_weights): read by the forward / backward-data launch
    wfwd: object = None
    wbwd: object = None
    mma: int = 0  # CV_MMA_* operand precision of this layer's GEMMs (cvhip.set_precision)

    def geom(self, n: int) -> cv_conv:
        m = self.mod
        return cv_conv(
            n, self.c_in, self.h_in, self.w_in, self.c_out, self.h_out, self.w_out,
            m.kernel_size[0], m.kernel_size[1], m.stride[0], m.padding[0], int(self.transposed), self.mma,
        )


@dataclass
class VaeSpec:
    in_ch: int
    H: int
    W: int
    d: int  # z_dim (per factor)
    enc: list
    heads: list  # [mu_c, logvar_c, mu_s, logvar_s] nn.Linear
    feat: tuple  # (C, H, W) of the flattened encoder output
    dec_lin: nn.Linear
    dec_bn: nn.BatchNorm1d
    unflat: tuple  # (C, H, W) of the decoder Linear output
    dec: list = field(default_factory=list)
    mma: int = 0  # CV_MMA_* of the linear layers (the convs carry their own, set together)

    @property
    def F(self) -> int:
        c, h, w = self.feat
        return c * h * w

    @property
    def bn_layers(self) -> list:
        return [c.bn for c in self.enc] + [self.dec_bn] + [c.bn for c in self.dec]


def _conv_out(h, k, s, p):
    return (h + 2 * p - k) // s + 1


def _convT_out(h, k, s, p, op):
    return (h - 1) * s - 2 * p + k + op


def vae_spec(vae: nn.Module, image_hw: int | None = None) -> VaeSpec:
    """Derive the layer plan from the module tree (the attribute names of the reference VAE)."""
    enc_mods = list(vae.encoder)
    in_ch = None
    for m in enc_mods:
        if isinstance(m, nn.Conv2d):
            in_ch = m.in_channels
            break
    # image size: VAE (k=3) is 28x28; VAE64 (k=4) is 64x64 (Linear(2048) fixes both)
    first = next(m for m in enc_mods if isinstance(m, nn.Conv2d))
    if image_hw is None:
        image_hw = 28 if first.kernel_size[0] == 3 else 64
    h = w = image_hw
    c = in_ch
    enc = []
    i = 0
    while i < len(enc_mods):
        m = enc_mods[i]
        if isinstance(m, nn.Conv2d):
            bn = enc_mods[i + 1]
            assert isinstance(bn, nn.BatchNorm2d) and isinstance(enc_mods[i + 2], nn.ReLU), "unexpected encoder"
            k, s, p = m.kernel_size[0], m.stride[0], m.padding[0]
            ho, wo = _conv_out(h, k, s, p), _conv_out(w, k, s, p)
            enc.append(ConvSpec(m, bn, True, False, c, h, w, m.out_channels, ho, wo))
            c, h, w = m.out_channels, ho, wo
            i += 3
        elif isinstance(m, nn.Flatten):
            i += 1
        else:
            raise NotImplementedError(f"encoder module {type(m).__name__} not supported by the HIP path")
    feat = (c, h, w)
    heads = [vae.mu_c, vae.logvar_c, vae.mu_s, vae.logvar_s]
    assert heads[0].in_features == c * h * w, "encoder output does not match the latent heads"
    dec_mods = list(vae.decoder)
    dec_lin, dec_bn = dec_mods[0], dec_mods[1]
    assert isinstance(dec_lin, nn.Linear) and isinstance(dec_bn, nn.BatchNorm1d)
    assert isinstance(dec_mods[2], nn.ReLU) and isinstance(dec_mods[3], nn.Unflatten)
    unflat = tuple(dec_mods[3].unflattened_size)
    c, h, w = unflat
    dec = []
    i = 4
    while i < len(dec_mods):
        m = dec_mods[i]
        assert isinstance(m, nn.ConvTranspose2d), f"unexpected decoder module {type(m).__name__}"
        bn = dec_mods[i + 1]
        act = dec_mods[i + 2]
        k, s, p, op = m.kernel_size[0], m.stride[0], m.padding[0], m.output_padding[0]
        ho, wo = _convT_out(h, k, s, p, op), _convT_out(w, k, s, p, op)
        relu = isinstance(act, nn.ReLU)
        if not relu:
            assert isinstance(act, nn.Sigmoid) and i + 3 == len(dec_mods), "Sigmoid must end the decoder"
        dec.append(ConvSpec(m, bn, relu, True, c, h, w, m.out_channels, ho, wo))
        c, h, w = m.out_channels, ho, wo
        i += 3
    assert (c, h, w) == (in_ch, image_hw, image_hw), "decoder output does not match the input shape"
    return VaeSpec(in_ch, image_hw, image_hw, vae.z_dim, enc, heads, feat, dec_lin, dec_bn, unflat, dec)


# ----------------------------------------------------------------------------- flat parameter arena


class ParamArena:
    """All parameters of a module as views into one flat fp32 buffer (+ a flat gradient buffer)."""

    def __init__(self, params: list, device, tight=()):
        self.params = list(params)
        self.device = torch.device(device)
        # every parameter starts on a 16-byte boundary (float4 loads); the gaps stay zero and get zero
        # gradients, so Adam leaves them at zero.  `tight`: parameters followed directly by the next one (a group
        # the kernels address as one tensor: the four head weights [4d][F] and the four head biases [4d], whose
        # d-element biases would otherwise be padded apart when d % 4 != 0)
        tight = {id(p) for p in tight}
        self.offset = {}
        o = 0
        for p in self.params:
            self.offset[id(p)] = (o, p.numel())
            o = o + p.numel() if id(p) in tight else (o + p.numel() + 3) & ~3
        self.numel = o
        self.flat = torch.zeros(o, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(o, dtype=torch.float32, device=self.device)
        with torch.no_grad():
            for p in self.params:
                o, n = self.offset[id(p)]
                self.flat[o:o + n].copy_(p.data.reshape(-1).to(self.device, torch.float32))
                p.data = self.flat[o:o + n].view_as(p)

    def valid(self) -> bool:
        base = self.flat.data_ptr()
        for p in self.params:
            o, n = self.offset[id(p)]
            if p.data_ptr() != base + 4 * o or p.device != self.device or p.dtype != torch.float32:
                return False
        return True

    def pview(self, p) -> torch.Tensor:
        o, n = self.offset[id(p)]
        return self.flat[o:o + n].view_as(p)

    def gview(self, p) -> torch.Tensor:
        o, n = self.offset[id(p)]
        return self.grad[o:o + n].view_as(p)

    def gptr(self, p) -> int:
        return self.grad.data_ptr() + 4 * self.offset[id(p)][0]

    def pptr(self, p) -> int:
        return self.flat.data_ptr() + 4 * self.offset[id(p)][0]


def vae_param_order(vae: nn.Module, spec: VaeSpec) -> list:
    """Arena order: encoder, the 4 head weights (contiguous [4d, F]), the 4 head biases, decoder."""
    order = []
    for c in spec.enc:
        order += [c.mod.weight, c.mod.bias, c.bn.weight, c.bn.bias]
    order += [h.weight for h in spec.heads] + [h.bias for h in spec.heads]
    order += [spec.dec_lin.weight, spec.dec_lin.bias, spec.dec_bn.weight, spec.dec_bn.bias]
    for c in spec.dec:
        order += [c.mod.weight, c.mod.bias, c.bn.weight, c.bn.bias]
    names = {id(p) for p in order}
    rest = [p for p in vae.parameters() if id(p) not in names]
    if rest:
        raise NotImplementedError("VAE has parameters outside the CLEAR-VAE topology")
    if any(p is None for p in order):
        raise NotImplementedError("conv/linear layers without bias or BatchNorm without affine")
    return order


def ensure_arena(vae: nn.Module, spec_fn=None):
    """Attach (or re-attach) a ParamArena + VaeSpec to `vae` on its current device."""
    arena = getattr(vae, "_cv_arena", None)
    if arena is not None and arena.valid():
        return arena
    spec = vae_spec(vae) if spec_fn is None else spec_fn(vae)
    dev = next(vae.parameters()).device
    if dev.type != "cuda":
        raise RuntimeError(
            "clear-vae_amd runs on MI355X (ROCm device 'cuda'); move the model with .to('cuda') first"
        )
    arena = ParamArena(vae_param_order(vae, spec), dev,
                       tight=[h.weight for h in spec.heads[:-1]] + [h.bias for h in spec.heads[:-1]])
    attach_packed(spec, dev)
    vae._cv_arena = arena
    vae._cv_spec = spec
    vae._cv_workspaces = {}
    _apply_precision(spec, getattr(vae, "_cv_precision", "fp32"))
    return arena


def _apply_precision(spec: VaeSpec, precision: str):
    if precision not in _lib.PRECISION:
        raise ValueError(f"precision must be one of {sorted(_lib.PRECISION)}, got {precision!r}")
    mma = _lib.PRECISION[precision]
    spec.mma = mma
    for c in spec.enc + spec.dec:
        c.mma = mma


def set_precision(vae: nn.Module, precision: str = "fp32"):
    """Operand precision of the model's conv / linear contractions on the HIP path: "fp32" (the
    reference's arithmetic, default) or "bf16" (BASELINE configs[4]: operands rounded to bf16 for
    v_mfma_f32_16x16x32_bf16, fp32 accumulation; activations, BatchNorm statistics, losses and Adam stay
    fp32, as do the image-facing first conv / last convT and the latent-side linears, LIN_MMA).  Takes effect at the next step: a fused engine built for the other precision rebuilds."""
    if precision not in _lib.PRECISION:
        raise ValueError(f"precision must be one of {sorted(_lib.PRECISION)}, got {precision!r}")
    vae._cv_precision = precision
    spec = getattr(vae, "_cv_spec", None)
    if spec is not None:
        _apply_precision(spec, precision)


def attach_packed(spec: VaeSpec, device):
    """Allocate the packed conv weights (one buffer) and the cv_conv_pack descriptors.

    Wg[tap][cb][cs] ("gather") serves Conv2d forward / ConvTranspose2d backward-data and
    Ws[tap][cs][cb] ("scatter") serves Conv2d backward-data / ConvTranspose2d forward, where
    cs, cb = weight.shape[0], weight.shape[1] (include/clearvae.h, cv_conv_pack)."""
    convs = spec.enc + spec.dec
    total = sum(2 * c.mod.weight.numel() for c in convs)
    buf = torch.empty(total, dtype=torch.float32, device=device)
    o = 0
    spec.pack_items = {"enc": [], "dec": []}
    for part, lst in (("enc", spec.enc), ("dec", spec.dec)):
        for c in lst:
            w = c.mod.weight
            k = w.numel()
            gat, sca = buf[o:o + k], buf[o + k:o + 2 * k]
            o += 2 * k
            c.wfwd, c.wbwd = (sca, gat) if c.transposed else (gat, sca)
            spec.pack_items[part].append(
                cv_conv_pack(w.data_ptr(), gat.data_ptr(), sca.data_ptr(), w.shape[0], w.shape[1], w.shape[2],
                             w.shape[3]))
    spec.packed = buf
    # the four heads as one [4d][F] weight, packed [F (storage order)][4d] for cv_heads_forward: the conv pack's
    # gather order with cs = 4d, cb = C and the pixels as taps
    C, Hh, Wh = spec.feat
    hw = spec.heads[0].weight
    spec.heads_wp = torch.empty(4 * spec.d * spec.F, dtype=torch.float32, device=device)
    spec.pack_items["enc"].append(cv_conv_pack(hw.data_ptr(), spec.heads_wp.data_ptr(), None, 4 * spec.d, C, Hh, Wh))


def pack_program(spec: VaeSpec, P: "Program", which: str = "all", zero=None):
    """Refresh the packed conv weights from the (arena) parameters: one launch; `zero` = [(tensor,
    bytes)] buffers cleared by the same launch.  which=None: no packing (the zeroing only)."""
    items = ([] if which is None else
             spec.pack_items["enc"] * (which != "dec") + spec.pack_items["dec"] * (which != "enc"))
    if items and zero:
        P.add("cv_pack_conv_weights_zero", struct_array(cv_conv_pack, items), len(items),
              ptr_array([t.data_ptr() for t, _ in zero]), (ctypes.c_size_t * len(zero))(*[nb for _, nb in zero]),
              len(zero))
    elif items:
        P.add("cv_pack_conv_weights", struct_array(cv_conv_pack, items), len(items))
    elif zero:
        P.add("cv_zero_many", ptr_array([t.data_ptr() for t, _ in zero]),
              (ctypes.c_size_t * len(zero))(*[nb for _, nb in zero]), len(zero))


# ----------------------------------------------------------------------------- BN plumbing


class BNView:
    """One BatchNorm layer: its fp64 stats slots in the workspace and cv_bn builders."""

    def __init__(self, mod: nn.Module, stat: torch.Tensor, gstat: torch.Tensor, count: int):
        self.mod = mod
        self.C = mod.num_features
        self.stat = stat  # [REPL, 2, C] float64
        self.gstat = gstat
        self.count = count
        if mod.momentum is None:
            raise NotImplementedError("BatchNorm(momentum=None) cumulative averaging is not supported")
        if not mod.affine or not mod.track_running_stats:
            raise NotImplementedError("BatchNorm without affine / running stats is not supported")

    # finalised-constant slots (Workspace.__init__): cfwd [4C], cbwd [5C] fp32 and a ticket pair
    cfwd: torch.Tensor | None = None
    cbwd: torch.Tensor | None = None
    ticket: int | None = None

    # Producer-side finalisation of the BN constants (cv_bn.ticket, include/clearvae.h): a GEMM-core
    # producer writes them from its last workgroup and consuming GEMMs load them instead of folding the
    # replica sums.  It pays only where both sides are GEMM-core launches (Workspace sets fin_fwd /
    # fin_bwd for those layers): stamped per-block timelines on the MNIST step put the consumer
    # prologues at 7-10 -> 3.5-4.5 us, while finalising for a narrow-kernel consumer only adds the
    # producer's last-workgroup tail (up to +20 us on a 1,568-workgroup launch).
    FINALISE = True
    fin_fwd = False
    fin_bwd = False

    def cv(self, train: bool) -> cv_bn:
        m = self.mod
        fin = train and self.ticket is not None and self.FINALISE
        return cv_bn(
            m.weight.data_ptr(), m.bias.data_ptr(), self.stat.data_ptr(), self.gstat.data_ptr(),
            m.running_mean.data_ptr(), m.running_var.data_ptr(), self.C, self.count, int(train), float(m.eps),
            self.cfwd.data_ptr() if fin and self.fin_fwd else None, self.cbwd.data_ptr() if fin and self.fin_bwd else None,
            self.ticket if fin and (self.fin_fwd or self.fin_bwd) else None,
        )


def operand(x, xf=XF_NONE, bn: cv_bn | None = None, y=None, nchw=0) -> cv_operand:
    o = cv_operand()
    o.x = x.data_ptr() if isinstance(x, torch.Tensor) else x
    o.y = (y.data_ptr() if isinstance(y, torch.Tensor) else y) if y is not None else None
    o.xf = xf
    o.nchw = nchw
    if bn is not None:
        o.bn = bn
    return o


def ep_none() -> cv_epilogue:
    e = cv_epilogue()
    e.stat_mode = STAT_NONE
    e.stat_div = 1
    return e


def ep_fwd(bnv: BNView) -> cv_epilogue:
    e = ep_none()
    e.stat_mode = STAT_FWD
    e.stat_out = bnv.stat.data_ptr()
    e.ebn = bnv.cv(True)  # the producer's last workgroup finalises this layer's constants
    return e


def ep_bwd(bnv: BNView, ey: torch.Tensor, relu: bool, stat_div: int = 1) -> cv_epilogue:
    e = ep_none()
    e.stat_mode = STAT_BWD
    e.stat_out = bnv.gstat.data_ptr()
    e.stat_div = stat_div
    e.ey = ey.data_ptr()
    e.ebn = bnv.cv(True)
    e.erelu = int(relu)
    return e


# ----------------------------------------------------------------------------- programs


_SIDE_STREAMS: dict = {}
# Weight-gradient calls on a second stream: off by default.  In a replayed graph every cross-stream edge
# costs ~10 us of idle time on both queues (rocprofv3 kernel trace of the MNIST step, round 2), and the
# overlapped GEMMs slow each other down (each grid already fills the chip), so one stream measured as fast
# or faster on both bench configs (MNIST 0.7015 vs 0.7046 ms, CelebA-MIM 6.46 vs 6.60 ms).
# CVHIP_SIDE_STREAM=1 restores the two-stream schedule.
SIDE_STREAM = os.environ.get("CVHIP_SIDE_STREAM", "0") == "1"

# Operand precision of the latent-side linear layers (the four heads and the decoder Linear) under either model
# precision: fp32.  Their fused kernels (cv_declinear.hip: cv_heads_forward / _backward,
# cv_decoder_input_forward / _backward) run v_mfma_f32_16x16x4_f32 only, and they are < 0.4 % of a VAE64 step's
# FLOPs, so precision="bf16" applies to the conv / convT contractions of the GEMM core alone; the DENSE fallback
# (batches the fused kernels do not serve) is given the same fp32 geometry so the arithmetic does not depend on
# the batch size.  oracle/cpu_ref.py `bf16=` restates exactly this split.
LIN_MMA = _lib.MMA_FP32


def _side_stream(device, k: int = 1) -> "torch.cuda.Stream":
    """Side stream k (>= 1) of the device: one ordered queue per k, shared by every program."""
    key = (torch.device(device).index, k)
    st = _SIDE_STREAMS.get(key)
    if st is None:
        st = _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return st


JOIN = "join"  # lane of an explicit join entry
HOST = "host"  # lane of a host-side call (no stream: e.g. selecting a launch workspace while the calls are enqueued)


class Program:
    """A fixed list of C-ABI calls (the stream is supplied at run time).

    Each call has a lane: 0 is the stream the program runs on; k >= 1 is side stream k.  A side call forks from the
    main stream after the main-stream calls issued before it (an event), calls of one side lane stay ordered among
    themselves, and the main stream joins every side lane it forked at the end of the program (or at an explicit
    join).  ``add_side`` puts the backward programs' weight-gradient GEMMs on side lane 1 (CVHIP_SIDE_STREAM=1), so
    they overlap the next layer's data-gradient GEMM instead of queueing behind it (both only read what the fork
    point has completed); ``extend(other, lane=k)`` runs a whole program on side lane k (CLEAR-MIM's estimator decoder
    forwards, cvhip/engine.py).  Host entries (lane HOST) call a Python function at enqueue time."""

    def __init__(self):
        self.calls = []  # (name, fn, args, lane)
        self.keep = []  # keep ctypes structs alive
        self._events = []
        self.join_at_end = True

    def _conv(self, args):
        conv = []
        for a in args:
            if isinstance(a, ctypes.Structure):
                self.keep.append(a)
                conv.append(ctypes.byref(a))
            elif isinstance(a, torch.Tensor):
                conv.append(a.data_ptr())
            else:
                conv.append(a)
        return conv

    def add(self, name: str, *args):
        self.calls.append((name, getattr(_lib.lib(), name), self._conv(args), 0))

    def add_side(self, name: str, *args):
        self.calls.append((name, getattr(_lib.lib(), name), self._conv(args), 1 if SIDE_STREAM else 0))

    def add_fork(self, name: str, *args):
        """A call on side lane 1 regardless of CVHIP_SIDE_STREAM (it forks from the main-stream calls before
        it; a later add_join, in this or a later program, joins it back)."""
        self.calls.append((name, getattr(_lib.lib(), name), self._conv(args), 1))

    def add_join(self, lanes=()):
        """The main stream waits here for everything issued on the side lanes so far (and on `lanes`: side lanes a
        C-ABI call of this or an earlier program put work on, e.g. cv_conv_backward_deferred_kpack_side)."""
        self.calls.append((JOIN, None, list(lanes), JOIN))

    def add_host(self, name: str, fn, *args):
        """fn(*args) on the host when the program is enqueued (eagerly, or while a graph is captured)."""
        self.calls.append((name, fn, list(args), HOST))

    def extend(self, other: "Program", lane: int | None = None):
        """Append other's calls; lane=k moves its stream calls onto side lane k."""
        if lane is None:
            self.calls += other.calls
        else:
            self.calls += [(nm, fn, a, lane if isinstance(ln, int) else ln) for nm, fn, a, ln in other.calls]
        self.keep += other.keep

    def run(self, stream: int | None = None, join: bool | None = None, timer: list | None = None):
        """join=False leaves the side lanes running past the end of the program (a later program's
        run joins them: each side lane is one ordered queue); graph capture needs a join before its end.
        timer (eager measurement only, bench.py): a list that receives (call index, start, end) timing
        events recorded around each call on the stream the call runs on."""
        try:
            self._run(stream, join, timer)
        except BaseException:
            # a queued NT-Xent phase (cv_ntxent_aux) whose flush this program did not reach holds this step's
            # pointers: drop it, so the next queue or served launch does not issue it
            _lib.lib().cv_ntxent_aux_discard()
            raise

    def _event(self, i):
        # (created on the first, eager run and reused by graph capture: the call sequence is fixed)
        while len(self._events) <= i:
            self._events.append(torch.cuda.Event())
        return self._events[i]

    def _run(self, stream, join, timer):
        s = _lib.stream_handle() if stream is None else stream
        main = torch.cuda.current_stream()
        if not any(c[3] for c in self.calls):
            for i, (name, fn, args, _) in enumerate(self.calls):
                if timer is not None:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(main)
                rc = fn(*args, s)
                if rc != 0:
                    _lib.check(rc, name)
                if timer is not None:
                    e1.record(main)
                    timer.append((i, e0, e1))
            return
        ev = 0
        forked = {}  # side lane -> forked since the main stream's last call (no new fork needed)
        active = []  # side lanes forked in this run, not yet joined

        def join_all(extra=()):
            nonlocal ev
            # (a join with no side lane forked in this run joins side lane 1: a fork left open by an earlier
            # program, join_at_end=False)
            for k in (sorted(set(active) | set(extra)) or [1]):
                e = self._event(ev)
                ev += 1
                e.record(_side_stream(main.device, k))
                main.wait_event(e)
            active.clear()
            forked.clear()

        for i, (name, fn, args, lane) in enumerate(self.calls):
            if lane == JOIN:
                join_all(args)
                continue
            if lane == HOST:
                fn(*args)
                continue
            if lane:
                side = _side_stream(main.device, lane)
                if not forked.get(lane):  # fork: the side lane waits for the main-stream work so far
                    e = self._event(ev)
                    ev += 1
                    e.record(main)
                    side.wait_event(e)
                    forked[lane] = True
                    if lane not in active:
                        active.append(lane)
                st, h = side, side.cuda_stream
            else:
                forked.clear()  # (main-stream work after this point: a later side call forks again)
                st, h = main, s
            if timer is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
            rc = fn(*args, h)
            if rc != 0:
                _lib.check(rc, name)
            if timer is not None:
                e1.record(st)
                timer.append((i, e0, e1))
        if (self.join_at_end if join is None else join) and active:
            join_all()


class DeferGroup:
    """Records of the deferred weight-gradient calls that one cv_step_reduce sums (include/clearvae.h,
    cv_wgrad_defer): a contiguous array the calls fill at enqueue time."""

    CAP = 24  # MAX_DEFER of cv_step_reduce

    def __init__(self):
        self.arr = (cv_wgrad_defer * self.CAP)()
        self.n = 0

    def next(self):
        if self.n >= self.CAP:
            raise RuntimeError("more than 24 deferred weight gradients in one cv_step_reduce")
        ref = ctypes.cast(ctypes.addressof(self.arr) + self.n * ctypes.sizeof(cv_wgrad_defer),
                          ctypes.POINTER(cv_wgrad_defer))
        self.n += 1
        return ref


def struct_array(ctype, items):
    arr = (ctype * len(items))(*items)
    return arr


def ptr_array(ptrs):
    return (ctypes.c_void_p * len(ptrs))(*ptrs)


# ----------------------------------------------------------------------------- workspace


class Workspace:
    """Device buffers of one batch size for one model (all NHWC fp32 unless noted)."""

    def __init__(self, spec: VaeSpec, n: int, device, with_grad: bool = True, encoder: bool = True):
        """encoder=False: no encoder activations (a workspace that only decodes a given z: CLEAR-MIM's estimator
        decoder forwards)."""
        self.spec, self.n, self.device = spec, n, device
        _lib.ensure_gemm_workspace(device)
        f32 = dict(dtype=torch.float32, device=device)
        d = spec.d
        self.y_enc = [torch.empty(n * c.h_out * c.w_out * c.c_out if encoder else 0, **f32) for c in spec.enc]
        self.heads = torch.empty(n, 4 * d, **f32)
        self.z = torch.empty(n, 2 * d, **f32)
        self.h = torch.empty(n, spec.dec_lin.out_features, **f32)
        self.ah = torch.empty(n, spec.dec_lin.out_features, **f32)
        self.y_dec = [torch.empty(n * c.h_out * c.w_out * c.c_out, **f32) for c in spec.dec]
        self.xhat = torch.empty(n, spec.in_ch, spec.H, spec.W, **f32)
        # fp64 statistics arena: per BN layer [REPL,2,C] forward + [REPL,2,C] backward, plus scalars
        bns = spec.bn_layers
        counts = [n * c.h_out * c.w_out for c in spec.enc] + [n] + [n * c.h_out * c.w_out for c in spec.dec]
        # (+ CV_TICKET_WORDS arrival counters per layer after the scalars: zeroed with the statistics)
        tw = (_lib.TICKET_WORDS + 1) // 2  # in 8-byte words
        tot = sum(2 * _lib.stat_repl(b.num_features) * 2 * b.num_features for b in bns) + 64 + tw * len(bns)
        self.stats = torch.zeros(tot, dtype=torch.float64, device=device)
        # finalised BN constants (written by each layer's producing launch, read by the GEMM prologues)
        r4 = lambda v: (v + 3) & ~3  # noqa: E731  (16-byte aligned slots)
        self.bn_consts = torch.zeros(sum(r4(4 * b.num_features) + r4(5 * b.num_features) for b in bns), **f32)
        self.bnv = []
        o = 0
        for b, cnt in zip(bns, counts):
            R = _lib.stat_repl(b.num_features)
            sz = R * 2 * b.num_features
            st = self.stats[o:o + sz].view(R, 2, b.num_features)
            gs = self.stats[o + sz:o + 2 * sz].view(R, 2, b.num_features)
            self.bnv.append(BNView(b, st, gs, cnt))
            o += 2 * sz
        self.scal = self.stats[o:o + 64]  # [0:REC_REPL] rec replicas (cv_output_loss), [32] mse work
        oc = 0
        for i, bv in enumerate(self.bnv):
            C = bv.C
            bv.cfwd = self.bn_consts[oc:oc + 4 * C]
            bv.cbwd = self.bn_consts[oc + r4(4 * C):oc + r4(4 * C) + 5 * C]
            oc += r4(4 * C) + r4(5 * C)
            bv.ticket = self.stats.data_ptr() + 8 * (o + 64 + tw * i)
        # interior layers: produced and consumed by GEMM-core launches in both directions (the layers
        # next to the image-facing convs and the BatchNorm1d are served by the narrow / BN kernels)
        self.bn_enc = self.bnv[: len(spec.enc)]
        self.bn_1d = self.bnv[len(spec.enc)]
        self.bn_dec = self.bnv[len(spec.enc) + 1:]
        nd = len(spec.dec)
        for i, bv in enumerate(self.bn_enc):
            bv.fin_fwd = i >= 1 and bv.C % 32 == 0
            bv.fin_bwd = bv.C % 32 == 0  # (layer 0: produced by a GEMM-core bwd-data, read by the edge wgrad)
        for j, bv in enumerate(self.bn_dec):
            bv.fin_fwd = j + 1 < nd and bv.C % 32 == 0  # (layer nd-2: read by the edge scatter / wgrad)
            bv.fin_bwd = j + 2 < nd and bv.C % 32 == 0
        self.rec = self.scal[0:_lib.REC_REPL]
        # the decoder layers' statistics and arrival tickets (contiguous: BatchNorm1d then the ConvT layers), for
        # forwards that reuse the encoder of the previous one (CLEAR-MIM's estimator updates)
        ne = len(spec.enc)
        d0 = sum(2 * _lib.stat_repl(b.num_features) * 2 * b.num_features for b in bns[:ne])
        self.dec_stats = self.stats[d0:o]
        self.dec_tickets = self.stats[o + 64 + tw * ne:o + 64 + tw * len(bns)]
        if with_grad:
            self.g_enc = [torch.empty(n * c.h_out * c.w_out * c.c_out, **f32) for c in spec.enc]
            self.dheads = torch.empty(n, 4 * d, **f32)
            self.dz = torch.zeros(n, 2 * d, **f32)
            self.gah = torch.empty(n, spec.dec_lin.out_features, **f32)
            self.g_dec = [torch.empty(n * c.h_out * c.w_out * c.c_out, **f32) for c in spec.dec]
            self.lse = torch.empty(2, 2 * n, **f32)  # contrastive row log-sum-exps (2 branches)
            self.losses = torch.zeros(8, **f32)
            # the multi-workgroup latent combine's KL partial slots + arrival ticket (zeroed once; left zeroed)
            self.comb_work = torch.zeros(int(_lib.lib().cv_latent_combine_workspace_bytes()) // 8 + 1,
                                         dtype=torch.float64, device=f32["device"])
            # cv_latent_combine_dz: KL slots, tickets and the dz contraction's slice tiles (zeroed once)
            self.comb_dz_work = torch.zeros(int(_lib.lib().cv_latent_combine_dz_workspace_bytes(n, d)) // 8 + 1,
                                            dtype=torch.float64, device=f32["device"])
            self.mi_work = torch.zeros(int(_lib.lib().cv_mi_workspace_bytes(n)) // 4 + 16, **f32)
            # split-K partial tiles of the weight-gradient GEMMs (one launch at a time on the stream)
            L = _lib.lib()
            C, Hh, Wh = spec.feat
            wb = [int(L.cv_conv_wgrad_workspace_bytes(ctypes.byref(c.geom(n)), 0)) for c in spec.enc + spec.dec]
            wb.append(int(L.cv_linear_wgrad_workspace_bytes(
                ctypes.byref(cv_linear(n, spec.F, 4 * d, Hh * Wh, C, 1, 0)), 0)))
            self.wg_bytes = max(wb + [16])
            self.wg_work = torch.empty(self.wg_bytes // 4, **f32)
            self._defer_work = {}  # deferred weight gradients: one partial-tile region per call

    def _wgrad_call(self, P: "Program", kind: str, geom, a, b, gw, gb, key, defer):
        """One weight-gradient call.  defer=None: reduced in place (shared split-K workspace).  defer=a
        DeferGroup: cv_*_backward_weight_deferred with its own workspace, its cv_wgrad_defer record in the
        group for the step's cv_step_reduce."""
        L = _lib.lib()
        if defer is None:
            if kind == "conv":
                P.add_side("cv_conv_backward_weight", geom, a, b, gw, gb, 0, self.wg_work, self.wg_bytes)
            else:
                P.add_side("cv_linear_backward_weight", geom, a, b, gw, gb, 0, self.wg_work, self.wg_bytes)
            return
        buf = self._defer_buf(kind, geom, key)
        name = "cv_conv_backward_weight_deferred" if kind == "conv" else "cv_linear_backward_weight_deferred"
        P.add(name, geom, a, b, gw, gb, buf, buf.numel() * 4, defer.next())

    def _defer_buf(self, kind: str, geom, key):
        L = _lib.lib()
        nb = int((L.cv_conv_wgrad_workspace_bytes if kind == "conv" else L.cv_linear_wgrad_workspace_bytes)(
            ctypes.byref(geom), 0))
        buf = self._defer_work.get(key)
        if buf is None or buf.numel() * 4 < nb:
            buf = self._defer_work[key] = torch.empty(max(nb, 16) // 4 + 4, dtype=torch.float32, device=self.device)
        return buf

    # cv_conv_backward_deferred: data and deferred weight gradient of a layer in one call (one launch for the
    # image-side ConvTranspose2d; CVHIP_FUSED_EDGE_BWD=0: the two calls)
    FUSED_EDGE_BWD = os.environ.get("CVHIP_FUSED_EDGE_BWD", "1") != "0"

    # deferred weight gradients of the interior layers on side stream 1 (cv_conv_backward_deferred_kpack_side), beside
    # the next layers' backward-data launches; set per workspace by the engine (single-process steps, CVHIP_WGRAD_LANE),
    # whose programs join side stream 1 before cv_step_reduce
    wgrad_side = False
    wgrad_side_first = False  # (also the decoder's first ConvTranspose2d, whose backward-data writes d(h))
    wgrad_lanes = 1  # side streams the weight gradients rotate over (1, 2, ...)
    _wside_next = 0

    def side_lanes(self):
        """The side lanes the weight gradients of this workspace's programs use (joined before cv_step_reduce)."""
        return list(range(1, self.wgrad_lanes + 1)) if self.wgrad_side else []

    def _conv_backward(self, P: "Program", geom, gout, wpacked, wkpack, gin, ep, xin, gw, key, defer):
        if defer is None or not self.FUSED_EDGE_BWD:
            P.add("cv_conv_backward_data_kpack", geom, gout, wpacked, wkpack, gin, ep)
            self._wgrad_call(P, "conv", geom, xin, gout, gw, None, key, defer)
            return
        buf = self._defer_buf("conv", geom, key)
        if self.wgrad_side and min(geom.c_in, geom.c_out) > 4:
            lane = 1 + self._wside_next % self.wgrad_lanes
            self._wside_next += 1
            P.add("cv_conv_backward_deferred_kpack_side", geom, gout, wpacked, wkpack, gin, ep, xin, gw, None, buf,
                  buf.numel() * 4, defer.next(), _side_stream(self.device, lane).cuda_stream)
            return
        P.add("cv_conv_backward_deferred_kpack", geom, gout, wpacked, wkpack, gin, ep, xin, gw, None, buf,
              buf.numel() * 4, defer.next())

    def _views(self, which) -> list:
        """BN layers by name ('all', 'enc', 'dec') or an explicit list of BNViews (a gradient bucket's)."""
        if isinstance(which, str):
            return {"all": self.bnv, "enc": self.bn_enc, "dec": [self.bn_1d] + self.bn_dec}[which]
        return list(which)

    def step_reduce_program(self, P: "Program", defer: "DeferGroup", param_grad, which="all",
                            running: bool = True, adam=None):
        """cv_step_reduce: the group's deferred weight gradients, the BN affine gradients of `which`
        layers and (running=True) their running statistics, in one launch.  adam = (params, grads, exp_avg,
        exp_avg_sq, numel, hyper, step, aux_counter): cv_step_reduce_adam, the optimizer step in the same
        launch."""
        views = self._views(which)
        bns = struct_array(cv_bn, [b.cv(True) for b in views])
        dg = ptr_array([param_grad(b.mod.weight) for b in views])
        db = ptr_array([param_grad(b.mod.bias) for b in views])
        nbt = ptr_array([b.mod.num_batches_tracked.data_ptr() for b in views]) if running else None
        if adam is not None:
            P.add("cv_step_reduce_adam", defer.arr, defer.n, bns, len(views), dg, db, int(running),
                  ctypes.c_float(float(views[0].mod.momentum)), nbt, *adam)
            return
        P.add("cv_step_reduce", defer.arr, defer.n, bns, len(views), dg, db, int(running),
              ctypes.c_float(float(views[0].mod.momentum)), nbt)

    # -- programs --------------------------------------------------------------------------
    def forward_program(self, x: torch.Tensor, train: bool, eps=None, seed: int = 0, offset=None,
                        output: str = "xhat", rec_scale=None) -> Program:
        """Encoder + heads + reparam + decoder (+ running statistics).  output: 'xhat'
        (cv_output_forward), 'loss' (cv_convt_output_loss: the last ConvT + cv_output_loss with the backward seed),
        'none' (statistics only)."""
        P = Program()
        if train:
            P.add("cv_zero", self.stats, self.stats.numel() * 8)
        drew = self.encoder_program(P, x, train, reparam=(eps, seed, offset))
        self.decoder_program(P, self.z, train, output, x, rec_scale, reparam=None if drew else (eps, seed, offset))
        if train:
            self.running_program(P, "all")
        return P

    # cv_heads_forward (cv_declinear.hip): the heads and the reparameterisation of their rows in one launch
    # (CVHIP_FUSED_HEADS_FWD=0: the DENSE split-K GEMM, the reparameterisation inside the decoder-input launch)
    FUSED_HEADS_FWD = os.environ.get("CVHIP_FUSED_HEADS_FWD", "1") != "0"

    def fused_heads_forward(self) -> bool:
        sp = self.spec
        C, Hh, Wh = sp.feat
        return (self.FUSED_HEADS_FWD and getattr(sp, "heads_wp", None) is not None
                and bool(_lib.lib().cv_heads_forward_supported(self.n, sp.F, C, sp.d)))

    def encoder_program(self, P: Program, x, train: bool, zero_heads: bool = True, reparam=None) -> bool:
        """Encoder + heads.  reparam = (eps, seed, offset): also draw z in the heads launch when the fused heads
        kernel serves this shape; returns True if it did (the caller then decodes z as given)."""
        sp, n = self.spec, self.n
        cur = None
        for li, c in enumerate(sp.enc):
            g = c.geom(n)
            if li == 0:
                op = operand(x, nchw=1)
            else:
                op = operand(cur, XF_BNRELU, self.bn_enc[li - 1].cv(train))
            ep = ep_fwd(self.bn_enc[li]) if train else ep_none()
            P.add("cv_conv_forward_kpack", g, op, c.wfwd, c.wbwd, c.mod.bias, self.y_enc[li], ep)
            cur = self.y_enc[li]
        # heads (Linear on the NCHW-flattened activation)
        C, Hh, Wh = sp.feat
        lin = cv_linear(n, sp.F, 4 * sp.d, Hh * Wh, C, 1, 0, LIN_MMA)
        if self.fused_heads_forward():
            eps, seed, offset = reparam if reparam is not None else (None, 0, None)
            P.add("cv_heads_forward", lin, cur, self.bn_enc[-1].cv(train), sp.heads_wp, sp.heads[0].bias.data_ptr(),
                  self.heads, eps.data_ptr() if eps is not None else None, ctypes.c_uint64(seed),
                  offset.data_ptr() if offset is not None else None, self.z if reparam is not None else None)
            return reparam is not None
        # split-K into a zeroed buffer
        if zero_heads:  # (else the caller zeroed it earlier in the same program)
            P.add("cv_zero", self.heads, self.heads.numel() * 4)
        P.add("cv_linear_forward", lin, operand(cur, XF_BNRELU, self.bn_enc[-1].cv(train)),
              sp.heads[0].weight.data_ptr(), sp.heads[0].bias.data_ptr(), self.heads, 1, ep_none())
        return False

    def reparam_program(self, P: Program, eps=None, seed: int = 0, offset=None):
        P.add("cv_reparam_forward", self.heads, self.n, self.spec.d, eps.data_ptr() if eps is not None else None,
              ctypes.c_uint64(seed), offset.data_ptr() if offset is not None else None, self.z, None)

    def running_sets_program(self, P: Program, sets):
        """The momentum updates of several forwards in one launch, in order: sets = [list of BNViews], the same
        layers in each (cv_bn_update_running_sets)."""
        views0 = sets[0]
        bns = struct_array(cv_bn, [b.cv(True) for views in sets for b in views])
        nbt = ptr_array([b.mod.num_batches_tracked.data_ptr() for b in views0])
        P.add("cv_bn_update_running_sets", bns, len(views0), len(sets), ctypes.c_float(float(views0[0].mod.momentum)),
              nbt)

    def running_program(self, P: Program, which="all", side: bool = False):
        """side=True: on the side stream (only where nothing re-zeroes the statistics before a join).  which: a
        name ('all', 'enc', 'dec') or an explicit list of BNViews (possibly of several workspaces)."""
        views = self._views(which)
        bns = struct_array(cv_bn, [b.cv(True) for b in views])
        nbt = ptr_array([b.mod.num_batches_tracked.data_ptr() for b in views])
        (P.add_side if side else P.add)("cv_bn_update_running", bns, len(views),
                                        ctypes.c_float(float(views[0].mod.momentum)), nbt)

    # cv_decoder_input_forward / _backward (cv_declinear.hip): the reparameterisation, the decoder Linear, its
    # BatchNorm1d and ReLU in one launch, and the mask + BN1d backward + Linear weight gradient in one launch
    # (CVHIP_FUSED_DECIN=0: the separate reparam / Linear / bn_apply and mask / weight-gradient launches)
    FUSED_DECIN = os.environ.get("CVHIP_FUSED_DECIN", "1") != "0"
    # CVHIP_DECIN_DRAW=1: the decoder-input launch draws z itself when the step has not (the CLEAR-MIM estimator
    # forwards); every one of its workgroups then redraws all n x 2d latents.  Default: one cv_reparam_forward
    # launch first (measured: 26.4 us for the drawing launch vs ~5 + 11.7 us)
    DECIN_DRAW = os.environ.get("CVHIP_DECIN_DRAW", "0") == "1"

    def decoder_input_geometry(self):
        sp = self.spec
        Cu, Hu, Wu = sp.unflat
        return cv_linear(self.n, 2 * sp.d, sp.dec_lin.out_features, 1, 0, Hu * Wu, Cu, LIN_MMA)

    def fused_decoder_input(self) -> bool:
        sp = self.spec
        return self.FUSED_DECIN and bool(_lib.lib().cv_decoder_input_supported(self.n, sp.d, sp.dec_lin.out_features))

    # cv_heads_backward (cv_declinear.hip): the heads' data and weight gradients with the last encoder block's
    # ReLU mask and BN backward sums in one launch (CVHIP_FUSED_HEADS=0: the DENSE backward-data GEMM and the
    # deferred split-K weight gradient)
    FUSED_HEADS = os.environ.get("CVHIP_FUSED_HEADS", "1") != "0"

    def fused_heads(self) -> bool:
        sp = self.spec
        C, Hh, Wh = sp.feat
        return self.FUSED_HEADS and bool(_lib.lib().cv_heads_backward_supported(self.n, sp.F, C, 4 * sp.d))

    # CVHIP_STATS_ONLY_OUT (default 1): a train-mode decoder pass with output 'none' (CLEAR-MIM's estimator forwards,
    # CLEAR-TC's discriminator forward) does not write the pre-BN image (0: it does, A/B)
    STATS_ONLY_OUT = os.environ.get("CVHIP_STATS_ONLY_OUT", "1") != "0"

    def decoder_program(self, P: Program, z, train: bool, output: str, x=None, rec_scale=None, reparam=None,
                        aux=None, aux_combine=None, aux_at=None, aux_in=None):
        """reparam = (eps, seed, offset): z is drawn from self.heads first (cv_reparam_forward, or inside the
        fused decoder-input launch); None: z is given.  aux: cv_ntxent_aux argument tuples, the i-th queued before
        the i-th decoder conv (its phase rides in that launch where served) and flushed right after it — or
        before the decoder conv aux_at[i] (the last one: the output-loss call, whose loss launch serves a gradient
        phase); aux_combine: cv_ntxent_aux_combine arguments attached to the first (the KL part of the latent
        combine); aux_in: cv_ntxent_aux arguments queued before the decoder-input launch (which serves it) and
        flushed after it."""
        sp, n = self.spec, self.n
        Cu, Hu, Wu = sp.unflat
        lin = cv_linear(n, 2 * sp.d, sp.dec_lin.out_features, 1, 0, Hu * Wu, Cu, LIN_MMA)
        if self.fused_decoder_input():
            if reparam is not None and not self.DECIN_DRAW:  # z drawn once, by its own launch
                eps, seed, offset = reparam
                P.add("cv_reparam_forward", self.heads, n, sp.d, eps.data_ptr() if eps is not None else None,
                      ctypes.c_uint64(seed), offset.data_ptr() if offset is not None else None, z, None)
                reparam = None
            eps, seed, offset = reparam if reparam is not None else (None, 0, None)
            if aux_in is not None:
                P.add("cv_ntxent_aux", *aux_in)
            P.add("cv_decoder_input_forward", lin, self.heads if reparam is not None else None,
                  eps.data_ptr() if eps is not None else None, ctypes.c_uint64(seed),
                  offset.data_ptr() if offset is not None else None, z, sp.dec_lin.weight, sp.dec_lin.bias,
                  self.bn_1d.cv(train), self.bn_1d.stat if train else None, self.h, self.ah)
            if aux_in is not None:
                P.add("cv_ntxent_aux_flush")
        else:
            if aux_in is not None:  # (no fused decoder-input launch to serve it: its own launch)
                P.add("cv_ntxent_aux", *aux_in)
                P.add("cv_ntxent_aux_flush")
            if reparam is not None:
                self.reparam_program(P, *reparam)
            ep = ep_fwd(self.bn_1d) if train else ep_none()
            P.add("cv_linear_forward", lin, operand(z), sp.dec_lin.weight, sp.dec_lin.bias, self.h, 0, ep)
            P.add("cv_bn_apply", self.bn_1d.cv(train), self.h, self.ah, n, sp.dec_lin.out_features, Hu * Wu, Cu, 1)
        cur = self.ah
        last = sp.dec[-1]
        hw = last.h_out * last.w_out
        at = {} if aux is None else {(aux_at[q] if aux_at is not None else q): q for q in range(len(aux))}
        for li, c in enumerate(sp.dec):
            g = c.geom(n)
            op = operand(cur) if li == 0 else operand(cur, XF_BNRELU, self.bn_dec[li - 1].cv(train))
            ep = ep_fwd(self.bn_dec[li]) if train else ep_none()
            q = at.get(li)
            if q is not None:
                P.add("cv_ntxent_aux", *aux[q])
                if q == 0 and aux_combine is not None:
                    P.add("cv_ntxent_aux_combine", *aux_combine)
            if li == len(sp.dec) - 1 and output == "loss":  # the last ConvT and the output / loss seed together
                assert train
                P.add("cv_convt_output_loss", g, op, c.wfwd, c.mod.bias, self.y_dec[li], ep, self.bn_dec[-1].cv(True), x,
                      self.xhat, self.rec, self.g_dec[-1], self.bn_dec[-1].gstat, rec_scale)
                if q is not None:
                    P.add("cv_ntxent_aux_flush")
                return
            # (a train-mode forward whose output is not wanted: the last ConvTranspose2d writes only its BatchNorm's
            # batch statistics, not the pre-BN image — cv_conv_forward with out = NULL, the edge scatter)
            stats_only = output == "none" and train and li == len(sp.dec) - 1 and self.STATS_ONLY_OUT
            P.add("cv_conv_forward_kpack", g, op, c.wfwd, c.wbwd, c.mod.bias, None if stats_only else self.y_dec[li],
                  ep)
            if q is not None:
                P.add("cv_ntxent_aux_flush")
            cur = self.y_dec[li]
        if output == "xhat":
            P.add("cv_output_forward", self.bn_dec[-1].cv(train), cur, n, sp.in_ch, hw, self.xhat)

    def decoder_backward_program(self, P: Program, param_grad, dz_out, zero_dz: bool = True, defer=None,
                                 aux_in=None, dz_later: bool = False):
        """From dv (= self.g_dec[-1], masked grad at the output BN, with its gstat filled) down to
        dz_out [n, 2d] (zeroed + accumulated) and the decoder parameter gradients.  aux_in: cv_ntxent_aux arguments
        queued before the decoder-input backward launch (which serves it) and flushed after it.  dz_later: the fused
        decoder-input backward leaves dz to the latent combine (cv_latent_combine_dz: deterministic) and writes only
        d(h) into gah."""
        sp, n = self.spec, self.n
        L = len(sp.dec)
        for li in range(L - 1, -1, -1):
            c = sp.dec[li]
            g = c.geom(n)
            gout = operand(self.g_dec[li], XF_BNBWD, self.bn_dec[li].cv(True), y=self.y_dec[li])
            if li > 0:
                ep = ep_bwd(self.bn_dec[li - 1], self.y_dec[li - 1], sp.dec[li - 1].relu)
                xin = operand(self.y_dec[li - 1], XF_BNRELU, self.bn_dec[li - 1].cv(True))
                self._conv_backward(P, g, gout, c.wbwd, c.wfwd, self.g_dec[li - 1], ep, xin,
                                    param_grad(c.mod.weight), ("dec", li), defer)
                continue
            elif defer is not None and self.wgrad_side and self.wgrad_side_first and self.FUSED_EDGE_BWD:
                # (the first ConvTranspose2d's weight gradient on the side stream too: beside the decoder-input
                # backward and the latent launches that follow)
                self._conv_backward(P, g, gout, c.wbwd, c.wfwd, self.gah, ep_none(), operand(self.ah),
                                    param_grad(c.mod.weight), ("dec", li), defer)
                continue
            else:
                P.add("cv_conv_backward_data_kpack", g, gout, c.wbwd, c.wfwd, self.gah, ep_none())
                xin = operand(self.ah)
            self._wgrad_call(P, "conv", g, xin, gout, param_grad(c.mod.weight), None, ("dec", li), defer)
        Cu, Hu, Wu = sp.unflat
        lin = cv_linear(n, 2 * sp.d, sp.dec_lin.out_features, 1, 0, Hu * Wu, Cu, LIN_MMA)
        if self.fused_decoder_input():  # gah <- d(h) in place, weight gradient, BN1d backward sums, dz
            if zero_dz:
                P.add("cv_zero", dz_out, dz_out.numel() * 4)
            if aux_in is not None:
                P.add("cv_ntxent_aux", *aux_in)
            P.add("cv_decoder_input_backward", lin, self.gah, self.h, self.bn_1d.cv(True), self.bn_1d.gstat,
                  self.z, param_grad(sp.dec_lin.weight), sp.dec_lin.weight, None if dz_later else dz_out)
            if aux_in is not None:
                P.add("cv_ntxent_aux_flush")
            return
        if aux_in is not None:  # (no fused decoder-input launch to serve it: its own launch)
            P.add("cv_ntxent_aux", *aux_in)
            P.add("cv_ntxent_aux_flush")
        else:
            P.add("cv_declinear_backward_weight", lin, self.gah, self.h, self.bn_1d.cv(True), self.bn_1d.gstat,
                  self.z, param_grad(sp.dec_lin.weight))
            gout = operand(self.gah, XF_BNBWD, self.bn_1d.cv(True), y=self.h)
        if zero_dz:  # (else the caller zeroed it earlier in the step)
            P.add("cv_zero", dz_out, dz_out.numel() * 4)
        P.add("cv_linear_backward_data", lin, gout, sp.dec_lin.weight, dz_out, 1, ep_none())

    def encoder_backward_program(self, P: Program, param_grad, dheads, x=None, dx=None, defer=None, heads=True,
                                 layers=None, chain=None):
        """From d(heads) [n, 4d] to the encoder / heads parameter gradients (and dx if asked).  A data-parallel
        step splits it in two programs at a layer boundary (heads=False and `layers`, the conv layers in
        backward order, for the second) so the first part's gradient bucket is reduced during the second.
        chain: a cv_latent_chain whose decoder-chain term the fused heads backward adds to dheads as it reads it
        (cv_heads_backward_chain; requires fused_heads())."""
        sp, n = self.spec, self.n
        C, Hh, Wh = sp.feat
        if heads and chain is not None:
            assert self.fused_heads()
            lin = cv_linear(n, sp.F, 4 * sp.d, Hh * Wh, C, 1, 0, LIN_MMA)
            P.add("cv_heads_backward_chain", lin, dheads, chain, sp.heads[0].weight, self.y_enc[-1],
                  self.bn_enc[-1].cv(True), self.g_enc[-1], self.bn_enc[-1].gstat, param_grad(sp.heads[0].weight),
                  param_grad(sp.heads[0].bias))
        elif heads and self.fused_heads():
            lin = cv_linear(n, sp.F, 4 * sp.d, Hh * Wh, C, 1, 0, LIN_MMA)
            P.add("cv_heads_backward", lin, dheads, sp.heads[0].weight, self.y_enc[-1], self.bn_enc[-1].cv(True),
                  self.g_enc[-1], self.bn_enc[-1].gstat, param_grad(sp.heads[0].weight), param_grad(sp.heads[0].bias))
        elif heads:
            lin = cv_linear(n, sp.F, 4 * sp.d, Hh * Wh, C, 1, 0, LIN_MMA)
            a_last = operand(self.y_enc[-1], XF_BNRELU, self.bn_enc[-1].cv(True))
            self._wgrad_call(P, "linear", lin, operand(dheads), a_last, param_grad(sp.heads[0].weight),
                             param_grad(sp.heads[0].bias), ("heads",), defer)
            ep = ep_bwd(self.bn_enc[-1], self.y_enc[-1], True, stat_div=Hh * Wh)
            P.add("cv_linear_backward_data", lin, operand(dheads), sp.heads[0].weight, self.g_enc[-1], 0, ep)
        for li in (range(len(sp.enc) - 1, -1, -1) if layers is None else layers):
            c = sp.enc[li]
            g = c.geom(n)
            gout = operand(self.g_enc[li], XF_BNBWD, self.bn_enc[li].cv(True), y=self.y_enc[li])
            if li > 0:
                ep = ep_bwd(self.bn_enc[li - 1], self.y_enc[li - 1], True)
                xin = operand(self.y_enc[li - 1], XF_BNRELU, self.bn_enc[li - 1].cv(True))
                if defer is not None and self.FUSED_EDGE_BWD:
                    # backward-data + deferred weight gradient in one call: one dual launch where the pair is
                    # served (cv_dual.hip)
                    self._conv_backward(P, g, gout, c.wbwd, c.wfwd, self.g_enc[li - 1], ep, xin,
                                        param_grad(c.mod.weight), ("enc", li), defer)
                    continue
                P.add("cv_conv_backward_data_kpack", g, gout, c.wbwd, c.wfwd, self.g_enc[li - 1], ep)
            else:
                if dx is not None:
                    P.add("cv_conv_backward_data", g, gout, c.wbwd, dx, ep_none())
                xin = operand(x, nchw=1)
            self._wgrad_call(P, "conv", g, xin, gout, param_grad(c.mod.weight), None, ("enc", li), defer)

    def bn_grads_program(self, P: Program, param_grad, which: str = "all", side: bool = False):
        views = {"all": self.bnv, "enc": self.bn_enc, "dec": [self.bn_1d] + self.bn_dec}[which]
        bns = struct_array(cv_bn, [b.cv(True) for b in views])
        dg = ptr_array([param_grad(b.mod.weight) for b in views])
        db = ptr_array([param_grad(b.mod.bias) for b in views])
        (P.add_side if side else P.add)("cv_bn_param_grads", bns, len(views), dg, db)
