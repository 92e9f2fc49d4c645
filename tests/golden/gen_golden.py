"""Generate the golden fixtures tests/golden/*.npz from the REAL reference (development container only).

Runs one real `CLEARVAETrainer._train` / `ClearMIMVAETrainer._train` / `ClearTCVAETrainer._train` /
`HierarchicalVAETrainer._train` (GVAE / ML-VAE) step of scotsun/clear-vae
(imported read-only from /root/reference/code, never copied) in float64 on the CPU, with:
  * weights from oracle.cpu_ref.det_state / det_mlp (numpy PCG64, so no weights are stored),
  * inputs from oracle.cpu_ref.det_inputs (seeded; a checksum of them is stored to catch drift),
  * the reparameterisation noise injected through torch.randn_like (vae.py:58, called for c then s
    in VAE.generate, vae.py:70-73) and the CLUB-S permutation through torch.randperm
    (mi_estimator.py:138), both patched only for the duration of the step; GVAE / ML-VAE draw the content
    noise group after group with torch.randn(n_g, d) (vae.py:207), which is fed the group-order rows of
    eps_c (oracle.cpu_ref.group_order_noise),
  * Tensor.cuda neutralised (L1OutUB.forward hardcodes .cuda(), mi_estimator.py:185).
The losses the trainer computes are captured by wrapping the names src.trainer imported
(vae_loss, contrastive_loss) and the estimator's forward.  Stored per case: scalars (fp64), the
latents, x_hat (small cases), per-tensor gradient norms, every small gradient in full and a fixed
256-element sample of each large one, the same for the parameters after the trainer's Adam step, BN
running statistics after the step's forwards, and (CLEAR-MIM) the 5 estimator learning losses.

Usage (here only — /root/reference does not exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
"""

from __future__ import annotations

import contextlib
import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/code"
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

from oracle import cpu_ref as R  # noqa: E402

SMALL = 2048  # gradients / params with at most this many elements are stored in full
NSAMPLE = 256

# name, arch, z, C, n, n_labels, mode, sim_fn, ps, estimator, store_xhat
CASES = [
    ("vae_n64_cosine_ps1", "VAE", 16, 1, 64, 10, "clear", "cosine", True, None, True),
    ("vae_n64_cosine_ps0", "VAE", 16, 1, 64, 10, "clear", "cosine", False, None, False),
    ("vae_n64_l2_ps1", "VAE", 16, 1, 64, 10, "clear", "l2", True, None, False),
    ("vae_n64_jeffrey_ps1", "VAE", 16, 1, 64, 10, "clear", "jeffrey", True, None, False),
    ("vae_n64_mahalanobis_ps1", "VAE", 16, 1, 64, 10, "clear", "mahalanobis", True, None, False),
    ("vae_n64_modl2_ps1", "VAE", 16, 1, 64, 10, "clear", "modified_l2", True, None, False),
    ("vae_n512_cosine_ps1", "VAE", 16, 1, 512, 10, "clear", "cosine", True, None, False),
    ("vae_n64_mim_club", "VAE", 16, 1, 64, 10, "mim", "cosine", None, "CLUBSample", False),
    ("vae_n64_mim_l1out", "VAE", 16, 1, 64, 10, "mim", "cosine", None, "L1OutUB", False),
    ("vae64_n16_cosine_ps1", "VAE64", 64, 3, 16, 4, "clear", "cosine", True, None, True),
    ("vae64_n16_mim_club", "VAE64", 64, 3, 16, 4, "mim", "cosine", None, "CLUBSample", False),
    ("vae_n64_tc", "VAE", 16, 1, 64, 10, "tc", "cosine", None, None, False),
    ("vae64_n16_tc", "VAE64", 64, 3, 16, 4, "tc", "cosine", None, None, False),
    # GVAE / ML-VAE (the estimator field names the group mode); l40: 32 samples over 40 labels, so
    # mostly singleton groups and gaps in the label values
    ("vae_n64_gvae", "VAE", 16, 1, 64, 10, "group", None, None, "GVAE", False),
    ("vae_n64_mlvae", "VAE", 16, 1, 64, 10, "group", None, None, "MLVAE", True),
    ("vae_n32_gvae_l40", "VAE", 16, 1, 32, 40, "group", None, None, "GVAE", False),
    ("vae64_n16_mlvae", "VAE64", 64, 3, 16, 4, "group", None, None, "MLVAE", False),
]

HP = {
    "VAE": {"temperature": 0.1, "alpha": 100.0, "beta": 1 / 8, "loc": 0, "scale": 1, "lambda": 3.0,
            "lr": 5e-4, "est_lr": 2e-3, "factor_lr": 1e-3},
    "VAE64": {"temperature": 0.1, "alpha": 100.0, "beta": 1 / 32, "loc": 0, "scale": 1, "lambda": 3.0,
              "lr": 3e-5, "est_lr": 2e-3, "factor_lr": 1e-3},
}


def sample_idx(name: str, numel: int) -> np.ndarray:
    seed = int.from_bytes(hashlib.sha256(name.encode()).digest()[:4], "little")
    return np.sort(np.random.default_rng(seed).choice(numel, NSAMPLE, replace=False))


def input_checksum(x, label, ec, es, perm) -> np.ndarray:
    return np.array([x.sum(), (x * x).sum(), label.sum(), ec.sum(), es.sum(), perm.sum()], dtype=np.float64)


@contextlib.contextmanager
def injected(noise: list, perm):
    """Patch the reference's two random draws and its hardcoded .cuda() for one step."""
    orig_randn_like, orig_randperm, orig_cuda = torch.randn_like, torch.randperm, torch.Tensor.cuda

    def randn_like(t, *a, **k):
        return noise.pop(0).to(t.dtype).reshape(t.shape).clone()

    def randperm(n, *a, **k):
        assert n == perm.numel()
        return perm.clone()

    torch.randn_like = randn_like
    torch.randperm = randperm
    torch.Tensor.cuda = lambda self, *a, **k: self
    try:
        yield
    finally:
        torch.randn_like, torch.randperm, torch.Tensor.cuda = orig_randn_like, orig_randperm, orig_cuda


def run_case(case):
    name, arch, z, C, n, nl, mode, sim_fn, ps, est_kind, store_xhat = case
    sys.path.insert(0, REF)
    import src.trainer as T  # noqa: E402
    from src.models import mi_estimator as MI  # noqa: E402
    from src.models.vae import VAE, VAE64  # noqa: E402

    hp = dict(HP[arch])
    hw = R.IMAGE[arch]
    x, label, ec, es, perm = R.det_inputs(n, C, hw, z, nl)
    sd = R.det_state(arch, z, C)
    torch.manual_seed(0)
    model = (VAE if arch == "VAE" else VAE64)(z, C).double()
    model.load_state_dict({k: torch.as_tensor(np.asarray(v)).clone() for k, v in sd.items()}, strict=True)
    model = model.double()
    rec = {"vae_loss": [], "contrastive": [], "mi_in": []}

    def vae_loss_rec(X_hat, X, **lp):
        out = orig_vae_loss(X_hat, X, **lp)
        rec["vae_loss"].append((X_hat.detach().clone(), {k: v.detach().clone() for k, v in lp.items()},
                                [float(o) for o in out]))
        return out

    def contrastive_rec(*a, **k):
        out = orig_contrastive(*a, **k)
        rec["contrastive"].append(float(out))
        return out

    orig_vae_loss, orig_contrastive = T.vae_loss, T.contrastive_loss
    T.vae_loss, T.contrastive_loss = vae_loss_rec, contrastive_rec
    noise = [torch.tensor(ec), torch.tensor(es)]
    extra = []
    X = torch.tensor(x, dtype=torch.float64)
    L = torch.tensor(label)
    out = {}
    try:
        opt = torch.optim.Adam(model.parameters(), lr=hp["lr"])
        if mode == "group":
            model.mode = est_kind  # VAE(..., group_mode=...) (trainer_utils.py:69-71)
            L_t = torch.tensor(label)
            sorted_rows = R.group_order_noise(label, torch.tensor(ec))
            sizes = [int((L_t == g).sum()) for g in torch.unique(L_t, sorted=True)]
            chunks = list(torch.split(sorted_rows, sizes))
            noise.pop(0)  # eps_c is consumed through torch.randn, group by group
            orig_randn, orig_decode = torch.randn, model.decode
            zs = []

            def randn(*size, **k):
                t = chunks.pop(0)
                assert tuple(t.shape) == tuple(size), (t.shape, size)
                return t.clone()

            def decode_rec(zz):
                zs.append(zz.detach().clone())
                return orig_decode(zz)

            model.decode = decode_rec
            hyper = {k: hp[k] for k in ("beta", "loc", "scale")}  # get_hierarchical_vae_trainer (:76-80)
            tr = T.HierarchicalVAETrainer(model, opt, hyper, 1, torch.device("cpu"))
            torch.randn = randn
            try:
                with injected(noise, torch.tensor(perm)):
                    tr._train([(X, L)], False, 0)
            finally:
                torch.randn = orig_randn
                del model.decode
            assert not chunks, "unconsumed group noise"
            out["z"] = zs[0].numpy()
            out["m"] = np.int64(len(sizes))
        elif mode == "clear":
            hyper = {k: hp[k] for k in ("temperature", "alpha", "beta", "loc", "scale")}
            hyper["ps"] = ps
            tr = T.CLEARVAETrainer(model, opt, sim_fn, hyper, 1, torch.device("cpu"))
            with injected(noise, torch.tensor(perm)):
                tr._train([(X, L)], False, 0)
        elif mode == "tc":
            # factor discriminator of get_cleartcvae_trainer (trainer_utils.py:133-138), deterministic weights
            d = z // 2
            disc = torch.nn.Sequential(torch.nn.Linear(z, z), torch.nn.ReLU(), torch.nn.Linear(z, 1),
                                       torch.nn.Sigmoid()).double()
            disc.load_state_dict({k: torch.as_tensor(v) for k, v in R.det_disc(z).items()}, strict=True)
            calls = []
            orig_disc_fwd = disc.forward

            def disc_rec(zin):
                o = orig_disc_fwd(zin)
                calls.append((zin.detach().clone(), o.detach().clone()))
                return o

            disc.forward = disc_rec
            gen = np.random.default_rng(6)
            a, b = gen.standard_normal((n, d)), gen.standard_normal((n, d))  # the second forward's noise
            extra.append((a, b))
            noise += [torch.tensor(a), torch.tensor(b)]
            fopt = torch.optim.Adam(disc.parameters(), lr=hp["factor_lr"])
            hyper = {k: hp[k] for k in ("temperature", "alpha", "beta", "loc", "scale", "lambda")}
            tr = T.ClearTCVAETrainer(model, disc, {"vae_optim": opt, "factor_optim": fopt}, sim_fn, hyper, 1,
                                     torch.device("cpu"))
            fl = []
            with injected(noise, torch.tensor(perm)):
                tr._train([(X, L)], False, 0, fl)
            assert len(calls) == 3  # d_score (VAE step), joint and marginal scores (factor step)
            dsc = calls[0][1]
            out["mi"] = np.float64(torch.relu(torch.log(dsc / (1 - dsc))).mean())
            out["z"] = calls[0][0].numpy()
            out["z2"] = calls[1][0].numpy()
            out["factor_loss"] = np.float64(fl[0])
            for k, v in disc.state_dict().items():
                out["disc_after__" + k] = v.numpy()
            for k, v in disc.named_parameters():
                out["disc_grad__" + k] = v.grad.detach().numpy()
            out["extra_noise"] = np.stack([np.stack(p) for p in extra])  # [1, 2, n, d]
        else:
            d = z // 2
            M = R.det_mlp(d, z)
            est = getattr(MI, est_kind)(d, d, z).double()
            est.load_state_dict({k: torch.as_tensor(v) for k, v in M.items()}, strict=True)
            orig_fwd = est.forward

            def fwd_rec(xs, ys):
                rec["mi_in"].append((xs.detach().clone(), ys.detach().clone()))
                return orig_fwd(xs, ys)

            est.forward = fwd_rec
            gen = np.random.default_rng(5)
            for _ in range(5):
                a, b = gen.standard_normal((n, d)), gen.standard_normal((n, d))
                extra.append((a, b))
                noise += [torch.tensor(a), torch.tensor(b)]
            eopt = torch.optim.Adam(est.parameters(), lr=hp["est_lr"])
            hyper = {k: hp[k] for k in ("temperature", "alpha", "beta", "loc", "scale", "lambda")}
            tr = T.ClearMIMVAETrainer(model, est, {"vae_optim": opt, "mi_estimator_optim": eopt}, sim_fn, hyper, 1,
                                      torch.device("cpu"))
            mi_l, mi_ll = [], []
            with injected(noise, torch.tensor(perm)):
                tr._train([(X, L)], False, 0, mi_l, mi_ll)
            out["mi"] = np.float64(mi_l[0])
            out["mi_learning"] = np.array(mi_ll, dtype=np.float64)
            zc, zs = rec["mi_in"][0]
            out["z"] = torch.cat([zc, zs], 1).numpy()
            for k, v in est.state_dict().items():
                out["est_after__" + k] = v.numpy()
            out["extra_noise"] = np.stack([np.stack(p) for p in extra])  # [5, 2, n, d]
        assert not noise, "unconsumed injected noise"
    finally:
        T.vae_loss, T.contrastive_loss = orig_vae_loss, orig_contrastive
        sys.path.remove(REF)

    X_hat, lp, (r_, kc, ks) = rec["vae_loss"][0]
    out.update(rec=np.float64(r_), kl_c=np.float64(kc), kl_s=np.float64(ks))
    if mode != "group":
        out["c_loss"] = np.float64(rec["contrastive"][0])
    if mode == "clear":
        out["s_loss_raw"] = np.float64(rec["contrastive"][1])
        out["s_loss"] = np.float64(rec["contrastive"][1] if ps else -rec["contrastive"][1])
    for k in ("mu_c", "logvar_c", "mu_s", "logvar_s"):
        out[k] = lp[k].numpy()
    if store_xhat:
        out["xhat"] = X_hat.numpy().astype(np.float32)
    out["anneal_w0"] = np.float64(hp["beta"] / 2)
    for pname, p in model.named_parameters():
        g = p.grad.detach().numpy().reshape(-1)
        out["gnorm__" + pname] = np.float64(np.linalg.norm(g))
        pa = p.detach().numpy().reshape(-1)
        if g.size <= SMALL:
            out["grad__" + pname] = g.copy()
            out["after__" + pname] = pa.copy()
        else:
            idx = sample_idx(pname, g.size)
            out["gidx__" + pname] = idx.astype(np.int64)
            out["grad__" + pname] = g[idx].copy()
            out["after__" + pname] = pa[idx].copy()
    for bname, b in model.named_buffers():
        out["buf__" + bname] = b.detach().numpy().copy()
    meta = dict(arch=arch, z=z, C=C, n=n, n_labels=nl, mode=mode, sim_fn=sim_fn, ps=ps, estimator=est_kind,
                hp=hp, torch=torch.__version__)
    out["meta"] = np.array(repr(meta))
    out["input_checksum"] = input_checksum(x, label, ec, es, perm)
    return name, out


def main():
    if not os.path.isdir(REF):
        raise SystemExit(f"{REF} not found: the golden fixtures are generated in the development container only")
    torch.set_num_threads(8)
    only = set(sys.argv[1:])
    for case in CASES:
        if only and case[0] not in only:
            continue
        name, out = run_case(case)
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **out)
        print(f"{name}: {os.path.getsize(path) / 1024:.1f} KiB  rec={float(out['rec']):.10g} "
              f"kl_c={float(out['kl_c']):.10g} c={float(out.get('c_loss', np.nan)):.10g}")


if __name__ == "__main__":
    main()
