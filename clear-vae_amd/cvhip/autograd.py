"""autograd.Function wrappers: the module-level (non-fused) HIP path.

These keep the reference's ``nn.Module`` / autograd contract (code/src/models/vae.py:48-102,
code/src/losses.py:41-137, code/src/models/mi_estimator.py:108-198): parameters receive ``.grad``
through PyTorch's AccumulateGrad, so user loops written against the reference (loss.backward();
optimizer.step()) keep working.  All arithmetic runs in libclearvae_hip.so; each forward gets its own
Workspace so several forwards may be outstanding before their backward.  The fused trainer step
(engine.py) issues the same kernels without autograd.
"""

from __future__ import annotations

import torch

from . import _lib, rng
from ._lib import GROUP, MI_CLUBSAMPLE, SIM, cv_mlp, cv_mlp_grad, cv_ntxent_branch
from .plan import Program, Workspace, ensure_arena, pack_program


def _require_gpu(*ts):
    for t in ts:
        if t is not None and isinstance(t, torch.Tensor) and t.device.type != "cuda":
            raise RuntimeError("clear-vae_amd: HIP kernels need tensors on the ROCm device ('cuda')")


def _f32c(t):
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def _grad_buffer(arena):
    return torch.zeros(arena.numel, dtype=torch.float32, device=arena.device)


def _views(arena, buf, params):
    out = []
    for p in params:
        o, n = arena.offset[id(p)]
        out.append(buf[o:o + n].view_as(p))
    return out


# ----------------------------------------------------------------------------- encoder


def encoder_params(vae):
    sp = vae._cv_spec
    ps = []
    for c in sp.enc:
        ps += [c.mod.weight, c.mod.bias, c.bn.weight, c.bn.bias]
    ps += [h.weight for h in sp.heads] + [h.bias for h in sp.heads]
    return ps


def decoder_params(vae):
    sp = vae._cv_spec
    ps = [sp.dec_lin.weight, sp.dec_lin.bias, sp.dec_bn.weight, sp.dec_bn.bias]
    for c in sp.dec:
        ps += [c.mod.weight, c.mod.bias, c.bn.weight, c.bn.bias]
    return ps


class EncodeFn(torch.autograd.Function):
    """x -> (mu_c, logvar_c, mu_s, logvar_s)   (VAE.encode, vae.py:48-50)."""

    @staticmethod
    def forward(ctx, x, vae, *params):
        arena = vae._cv_arena
        sp = vae._cv_spec
        train = vae.training
        xc = _f32c(x)
        ws = Workspace(sp, xc.shape[0], xc.device, with_grad=True)
        P = Program()
        if train:
            P.add("cv_zero", ws.stats, ws.stats.numel() * 8)
        pack_program(sp, P, "enc")
        ws.encoder_program(P, xc, train)
        if train:
            ws.running_program(P, "enc")
        P.run()
        ctx.ws, ctx.vae, ctx.train = ws, vae, train
        ctx.save_for_backward(xc)
        d = sp.d
        h = ws.heads
        return h[:, 0:d], h[:, d:2 * d], h[:, 2 * d:3 * d], h[:, 3 * d:4 * d]

    @staticmethod
    def backward(ctx, g_mu_c, g_lv_c, g_mu_s, g_lv_s):
        if not ctx.train:
            raise NotImplementedError("backward through eval-mode BatchNorm is not supported by the HIP path")
        ws, vae = ctx.ws, ctx.vae
        (xc,) = ctx.saved_tensors
        sp = vae._cv_spec
        arena = vae._cv_arena
        d = sp.d
        dheads = torch.zeros(ws.n, 4 * d, dtype=torch.float32, device=xc.device)
        for k, g in enumerate((g_mu_c, g_lv_c, g_mu_s, g_lv_s)):
            if g is not None:
                dheads[:, k * d:(k + 1) * d] = g
        gbuf = _grad_buffer(arena)
        base = gbuf.data_ptr()

        def pg(p):
            return base + 4 * arena.offset[id(p)][0]

        need_dx = ctx.needs_input_grad[0]
        dx = None
        if need_dx:
            dx = torch.empty(ws.n, sp.H, sp.W, sp.in_ch, dtype=torch.float32, device=xc.device)
        P = Program()
        ws.encoder_backward_program(P, pg, dheads, x=xc, dx=dx)
        ws.bn_grads_program(P, pg, "enc")
        P.run()
        grads = _views(arena, gbuf, encoder_params(vae))
        if dx is not None:
            dx = dx.permute(0, 3, 1, 2).contiguous() if sp.in_ch > 1 else dx.view(ws.n, 1, sp.H, sp.W)
        return (dx, None, *grads)


class DecodeFn(torch.autograd.Function):
    """z -> xhat   (VAE.decode, vae.py:52-54)."""

    @staticmethod
    def forward(ctx, z, vae, *params):
        sp = vae._cv_spec
        train = vae.training
        zc = _f32c(z)
        ws = Workspace(sp, zc.shape[0], zc.device, with_grad=True)
        ws.z = zc
        P = Program()
        if train:
            P.add("cv_zero", ws.stats, ws.stats.numel() * 8)
        pack_program(sp, P, "dec")
        ws.decoder_program(P, zc, train, "xhat")
        if train:
            ws.running_program(P, "dec")
        P.run()
        ctx.ws, ctx.vae, ctx.train = ws, vae, train
        return ws.xhat

    @staticmethod
    def backward(ctx, g_xhat):
        if not ctx.train:
            raise NotImplementedError("backward through eval-mode BatchNorm is not supported by the HIP path")
        ws, vae = ctx.ws, ctx.vae
        sp = vae._cv_spec
        arena = vae._cv_arena
        gbuf = _grad_buffer(arena)
        base = gbuf.data_ptr()

        def pg(p):
            return base + 4 * arena.offset[id(p)][0]

        last = sp.dec[-1]
        P = Program()
        P.add("cv_output_backward", ws.bn_dec[-1].cv(True), ws.y_dec[-1], ws.xhat, _f32c(g_xhat), ws.n, sp.in_ch,
              last.h_out * last.w_out, ws.g_dec[-1], ws.bn_dec[-1].gstat)
        dz = torch.empty(ws.n, 2 * sp.d, dtype=torch.float32, device=ws.xhat.device)
        ws.decoder_backward_program(P, pg, dz)
        ws.bn_grads_program(P, pg, "dec")
        P.run()
        grads = _views(arena, gbuf, decoder_params(vae))
        return (dz, None, *grads)


class SampleFn(torch.autograd.Function):
    """z = mu + eps * exp(logvar / 2)   (VAE.sample, vae.py:56-60)."""

    @staticmethod
    def forward(ctx, mu, logvar):
        mu_c, lv_c = _f32c(mu), _f32c(logvar)
        z = torch.empty_like(mu_c)
        eps = rng.next_noise()
        if eps is not None:
            eps = _f32c(eps.to(mu_c.device))
            assert eps.shape == mu_c.shape, "injected noise shape mismatch"
        seed, off = rng.offset_tensor(mu_c.device)
        _lib.call("cv_sample_forward", mu_c.data_ptr(), lv_c.data_ptr(), mu_c.numel(),
                  eps.data_ptr() if eps is not None else None, seed, off.data_ptr(), z.data_ptr(),
                  _lib.stream_handle())
        ctx.save_for_backward(mu_c, z)
        return z

    @staticmethod
    def backward(ctx, dz):
        mu_c, z = ctx.saved_tensors
        dmu = torch.empty_like(mu_c)
        dlv = torch.empty_like(mu_c)
        _lib.call("cv_sample_backward", mu_c.data_ptr(), z.data_ptr(), _f32c(dz).data_ptr(), mu_c.numel(),
                  dmu.data_ptr(), dlv.data_ptr(), 0, _lib.stream_handle())
        return dmu, dlv


# ----------------------------------------------------------------------------- group evidence


def _group_offsets(n: int, d: int):
    """int32 offsets of m / order / start and the fp32 offset of the group rows in a cv_group_forward
    workspace (include/clearvae.h)."""
    order = 16 + 2 * n
    start = 16 + 3 * n
    rows = ((64 + 16 * n + 4) + 15) // 16 * 4
    return order, start, rows


class GroupEvidenceFn(torch.autograd.Function):
    """accumulate_group_evidence (vae.py:159-190): the group rows (mu_g, logvar_g) [m, d], segmented by
    label on the device (cv_group_forward).  `meta` (a dict) receives the groups as the reference's
    {label: member indices} dict; building it is the one host read of the call."""

    @staticmethod
    def forward(ctx, mu_c, logvar_c, label, mode, meta):
        if mode not in GROUP:
            raise NotImplementedError("only support using MLVAE or GVAE")
        mu, lv = _f32c(mu_c), _f32c(logvar_c)
        lab = label.reshape(-1).to(device=mu.device, dtype=torch.int64).contiguous()
        n, d = mu.shape
        work = torch.zeros(int(_lib.lib().cv_group_workspace_bytes(n, d)) // 4 + 4, dtype=torch.float32,
                           device=mu.device)
        _lib.call("cv_group_forward", GROUP[mode], mu.data_ptr(), lv.data_ptr(), d, lab.data_ptr(), n, d,
                  work.data_ptr(), None, None, None, 0, None, 0, 0, None, None, _lib.stream_handle())
        o_order, o_start, o_rows = _group_offsets(n, d)
        iw = work.view(torch.int32)
        host = torch.cat([iw[:1], iw[o_order:o_order + n], iw[o_start:o_start + n + 1]]).cpu()
        m = int(host[0])
        order, start = host[1:1 + n], host[1 + n:]
        lab_h = lab.cpu()
        order_d = iw[o_order:o_order + n].long()
        meta["groups"] = {int(lab_h[int(order[int(start[g])])]): order_d[int(start[g]):int(start[g + 1])]
                          for g in range(m)}
        rows = work[o_rows:o_rows + n * 2 * d].view(n, 2 * d)
        ctx.save_for_backward(mu, lv, work)
        ctx.meta = (GROUP[mode], n, d, m)
        return rows[:m, :d].clone(), rows[:m, d:].clone()

    @staticmethod
    def backward(ctx, g_mu, g_lv):
        mu, lv, work = ctx.saved_tensors
        mode, n, d, m = ctx.meta
        gm = _f32c(g_mu) if g_mu is not None else None
        gl = _f32c(g_lv) if g_lv is not None else None
        dmu = torch.empty(n, d, dtype=torch.float32, device=mu.device)
        dlv = torch.empty_like(dmu)
        _lib.call("cv_group_evidence_backward", mode, mu.data_ptr(), lv.data_ptr(), d, work.data_ptr(), n, d,
                  gm.data_ptr() if gm is not None else None, gl.data_ptr() if gl is not None else None,
                  dmu.data_ptr(), dlv.data_ptr(), d, _lib.stream_handle())
        return dmu, dlv, None, None, None


# ----------------------------------------------------------------------------- losses


def _rows(t):
    """(tensor, row stride) for a 2-D fp32 tensor whose rows may be strided (heads views)."""
    if t.dtype != torch.float32 or t.dim() != 2 or t.stride(1) != 1:
        t = _f32c(t)
    return t, t.stride(0)


class VaeLossFn(torch.autograd.Function):
    """(rec, kl_c, kl_s) of vae_loss (losses.py:41-50)."""

    @staticmethod
    def forward(ctx, xhat, x, mu_c, mu_s, lv_c, lv_s):
        xh, xx = _f32c(xhat), _f32c(x)
        n = xh.shape[0]
        out = torch.zeros(3, dtype=torch.float32, device=xh.device)
        work = torch.zeros(1, dtype=torch.float64, device=xh.device)
        s = _lib.stream_handle()
        _lib.call("cv_mse_sum", xh.data_ptr(), xx.data_ptr(), n, xh.numel() // n, out.data_ptr(), None, None,
                  work.data_ptr(), s)
        mc, ldc = _rows(mu_c)
        lc, _ = _rows(lv_c)
        ms, lds = _rows(mu_s)
        ls, _ = _rows(lv_s)
        assert lc.stride(0) == ldc and ls.stride(0) == lds
        # (each KL over its own rows: GVAE / ML-VAE pass the m group rows as mu_c / logvar_c)
        assert lc.shape == mc.shape and ls.shape == ms.shape
        _lib.call("cv_kl", mc.data_ptr(), lc.data_ptr(), ldc, mc.shape[0], mc.shape[1], out.data_ptr() + 4, None,
                  None, None, 0, 0, s)
        _lib.call("cv_kl", ms.data_ptr(), ls.data_ptr(), lds, ms.shape[0], ms.shape[1], out.data_ptr() + 8, None,
                  None, None, 0, 0, s)
        ctx.save_for_backward(xh, xx, mc, lc, ms, ls)
        return out[0], out[1], out[2]

    @staticmethod
    def backward(ctx, g_rec, g_kc, g_ks):
        xh, xx, mc, lc, ms, ls = ctx.saved_tensors
        n = xh.shape[0]
        s = _lib.stream_handle()
        res = [None] * 6
        if g_rec is not None and ctx.needs_input_grad[0]:
            g = _f32c(g_rec.reshape(1))
            dxh = torch.empty_like(xh)
            _lib.call("cv_mse_sum", xh.data_ptr(), xx.data_ptr(), n, xh.numel() // n, None, g.data_ptr(),
                      dxh.data_ptr(), None, s)
            res[0] = dxh
        for (m, l, gk, im, il) in ((mc, lc, g_kc, 2, 4), (ms, ls, g_ks, 3, 5)):
            if gk is None or not (ctx.needs_input_grad[im] or ctx.needs_input_grad[il]):
                continue
            g = _f32c(gk.reshape(1))
            dm = torch.empty(m.shape, dtype=torch.float32, device=m.device)
            dl = torch.empty_like(dm)
            _lib.call("cv_kl", m.data_ptr(), l.data_ptr(), m.stride(0), m.shape[0], m.shape[1], None, g.data_ptr(),
                      dm.data_ptr(), dl.data_ptr(), dm.stride(0), 0, s)
            res[im], res[il] = dm, dl
        return tuple(res)


class ContrastiveFn(torch.autograd.Function):
    """contrastive_loss(mu, logvar, label, sim_fn, temperature, "snn_loss", ps) (losses.py:98-137)."""

    @staticmethod
    def forward(ctx, mu, logvar, label, sim_fn, temperature, ps):
        if sim_fn not in SIM:
            raise ValueError("unimplemented similarity measure.")
        m, ld = _rows(mu)
        if logvar is not None:
            l_ = logvar if (logvar.dtype == torch.float32 and logvar.stride(0) == ld and logvar.stride(1) == 1) \
                else None
            if l_ is None:
                m = _f32c(mu)
                ld = m.stride(0)
                l_ = _f32c(logvar)
                assert l_.stride(0) == ld
        else:
            l_ = None
        lab = label.reshape(-1).to(torch.int64).contiguous()
        n, d = m.shape
        lse = torch.empty(2 * n, dtype=torch.float32, device=m.device)
        loss = torch.empty((), dtype=torch.float32, device=m.device)
        br = cv_ntxent_branch(m.data_ptr(), l_.data_ptr() if l_ is not None else None, ld, int(bool(ps)), None, None,
                              0, None, 1.0, loss.data_ptr(), lse.data_ptr())
        _lib.call("cv_ntxent", br, 1, lab.data_ptr(), n, d, SIM[sim_fn], float(temperature), 2, 0,
                  _lib.stream_handle())
        ctx.save_for_backward(m, l_ if l_ is not None else m, lab, lse)
        ctx.meta = (ld, SIM[sim_fn], float(temperature), int(bool(ps)), l_ is not None)
        return loss

    @staticmethod
    def backward(ctx, g):
        m, l_, lab, lse = ctx.saved_tensors
        ld, sim, tau, ps, has_lv = ctx.meta
        n, d = m.shape
        dmu = torch.empty(n, d, dtype=torch.float32, device=m.device)
        dlv = torch.empty(n, d, dtype=torch.float32, device=m.device)
        gg = _f32c(g.reshape(1))
        br = cv_ntxent_branch(m.data_ptr(), l_.data_ptr() if has_lv else None, ld, ps, dmu.data_ptr(),
                              dlv.data_ptr(), d, gg.data_ptr(), 1.0, None, lse.data_ptr())
        _lib.call("cv_ntxent", br, 1, lab.data_ptr(), n, d, sim, tau, 1, 0, _lib.stream_handle())
        return dmu, (dlv if has_lv else None), None, None, None, None


# ----------------------------------------------------------------------------- MI estimators


def mlp_struct(est) -> cv_mlp:
    """cv_mlp over an estimator's p_mu / p_logvar Sequentials (mi_estimator.py:111-122)."""
    l1, l2 = est.p_mu[0], est.p_mu[2]
    l3, l4 = est.p_logvar[0], est.p_logvar[2]
    for t in (l1.weight, l2.weight, l3.weight, l4.weight):
        if not t.is_contiguous() or t.dtype != torch.float32:
            raise RuntimeError("estimator weights must be contiguous fp32")
    return cv_mlp(l1.weight.data_ptr(), l1.bias.data_ptr(), l2.weight.data_ptr(), l2.bias.data_ptr(),
                  l3.weight.data_ptr(), l3.bias.data_ptr(), l4.weight.data_ptr(), l4.bias.data_ptr(),
                  l1.in_features, l1.out_features, l2.out_features)


def est_params(est):
    l1, l2 = est.p_mu[0], est.p_mu[2]
    l3, l4 = est.p_logvar[0], est.p_logvar[2]
    return [l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias, l4.weight, l4.bias]


class MIUpperBoundFn(torch.autograd.Function):
    """CLUBSample.forward / L1OutUB.forward (mi_estimator.py:133-143, 170-191)."""

    @staticmethod
    def forward(ctx, x, y, est, kind, *params):
        xx, yy = _f32c(x), _f32c(y)
        n = xx.shape[0]
        mlp = mlp_struct(est)
        work = torch.zeros(int(_lib.lib().cv_mi_workspace_bytes(n)) // 4 + 16, dtype=torch.float32,
                           device=xx.device)
        out = torch.empty((), dtype=torch.float32, device=xx.device)
        perm = None
        if kind == MI_CLUBSAMPLE:
            perm = rng.next_perm()
            if perm is not None:
                perm = perm.to(device=xx.device, dtype=torch.int64).contiguous()
        seed, off = rng.offset_tensor(xx.device)
        _lib.call("cv_mi_forward", kind, mlp, xx.data_ptr(), xx.stride(0), yy.data_ptr(), yy.stride(0), n,
                  perm.data_ptr() if perm is not None else None, seed, off.data_ptr(), work.data_ptr(),
                  out.data_ptr(), _lib.stream_handle())
        ctx.save_for_backward(xx, yy, work)
        ctx.est, ctx.kind, ctx.mlp = est, kind, mlp
        return out

    @staticmethod
    def backward(ctx, g):
        xx, yy, work = ctx.saved_tensors
        n, dxw = xx.shape
        gg = _f32c(g.reshape(1))
        dx = torch.empty_like(xx)
        dy = torch.empty_like(yy)
        params = est_params(ctx.est)
        gb = [torch.zeros_like(p) for p in params]
        G = cv_mlp_grad(*[t.data_ptr() for t in gb])
        _lib.call("cv_mi_backward", ctx.kind, ctx.mlp, xx.data_ptr(), xx.stride(0), yy.data_ptr(), yy.stride(0), n,
                  work.data_ptr(), gg.data_ptr(), 1.0, dx.data_ptr(), dy.data_ptr(), dxw, 0, G, None, None, None,
                  0, _lib.stream_handle())
        return (dx, dy, None, None, *gb)


class LearningLossFn(torch.autograd.Function):
    """learning_loss = -loglikeli (mi_estimator.py:129-131, 145-146, 193-198)."""

    @staticmethod
    def forward(ctx, x, y, est, *params):
        xx, yy = _f32c(x), _f32c(y)
        n = xx.shape[0]
        mlp = mlp_struct(est)
        ps = est_params(est)
        gb = [torch.empty_like(p) for p in ps]
        G = cv_mlp_grad(*[t.data_ptr() for t in gb])
        out = torch.empty((), dtype=torch.float32, device=xx.device)
        work = torch.zeros(int(_lib.lib().cv_mi_workspace_bytes(n)) // 4 + 16, dtype=torch.float32,
                           device=xx.device)
        _lib.call("cv_mi_learning_step", mlp, xx.data_ptr(), xx.stride(0), yy.data_ptr(), yy.stride(0), n,
                  work.data_ptr(), out.data_ptr(), G, None, None, None, None, 0, None, None, _lib.stream_handle())
        ctx.gb = gb
        ctx.xy_grad = (x.requires_grad, y.requires_grad)
        return out

    @staticmethod
    def backward(ctx, g):
        if any(ctx.xy_grad):
            raise NotImplementedError("learning_loss gradients w.r.t. its inputs (the reference detaches z)")
        gs = [t * g for t in ctx.gb]
        return (None, None, None, *gs)
