"""Golden fixtures (tests/golden/*.npz, made by tests/golden/gen_golden.py from the real reference) and
the oracle's restatement of the same step, shared by the CPU oracle-pinning test and the GPU parity
test.  Test infrastructure only."""

from __future__ import annotations

import ast
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def names() -> list:
    # the training-step fixtures (vae*_*.npz); resize_pil.npz and supcon.npz have their own tests
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f.startswith("vae"))


def load(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        fx = {k: z[k] for k in z.files}
    fx["meta"] = ast.literal_eval(str(fx["meta"]))
    return fx


def inputs(fx: dict):
    """The case's deterministic inputs (oracle.cpu_ref.det_inputs), checked against the stored checksum."""
    from oracle import cpu_ref as R

    m = fx["meta"]
    x, label, ec, es, perm = R.det_inputs(m["n"], m["C"], R.IMAGE[m["arch"]], m["z"], m["n_labels"])
    ck = np.array([x.sum(), (x * x).sum(), label.sum(), ec.sum(), es.sum(), perm.sum()], dtype=np.float64)
    assert np.allclose(ck, fx["input_checksum"], rtol=1e-12, atol=0), "input generator drifted from the fixtures"
    return x, label, ec, es, perm


def hyper(fx: dict) -> dict:
    m = fx["meta"]
    hp = dict(m["hp"])
    if m["mode"] == "clear":
        hp["ps"] = m["ps"]
    return hp


def oracle_step(fx: dict, dtype=torch.float64) -> dict:
    """One trainer step of the oracle (oracle/cpu_ref.py) on the fixture's case, in the fixture's keys."""
    from oracle import cpu_ref as R

    m = fx["meta"]
    arch, mode = m["arch"], m["mode"]
    x, label, ec, es, perm = inputs(fx)
    hp = hyper(fx)
    P = R.to_torch(R.det_state(arch, m["z"], m["C"]), dtype)
    X, L = torch.tensor(x, dtype=dtype), torch.tensor(label)
    Ec, Es = torch.tensor(ec, dtype=dtype), torch.tensor(es, dtype=dtype)
    out = {}
    if mode == "group":  # GVAE / ML-VAE: the content noise in group order (gen_golden.py)
        o = R.group_step(P, X, L, R.group_order_noise(label, Ec), Es, arch, hp, m["estimator"])
        out["z"] = o["z"].detach().numpy()
        out["m"] = o["m"]
    elif mode == "clear":
        o = R.clear_step(P, X, L, Ec, Es, arch, hp, m["sim_fn"])
        out["s_loss"] = float(o["s_loss"].detach())
    elif mode == "tc":
        D = R.to_torch(R.det_disc(m["z"]), dtype)
        o = R.tc_step(P, D, X, L, Ec, Es, arch, hp, m["sim_fn"])
        out["mi"] = float(o["mi"].detach())
        out["z"] = o["z"].detach().numpy()
    else:
        M = R.to_torch(R.det_mlp(m["z"] // 2, m["z"]), dtype)
        o = R.mim_step(P, M, X, L, Ec, Es, torch.tensor(perm), arch, hp, m["estimator"], m["sim_fn"])
        out["mi"] = float(o["mi"].detach())
        out["z"] = o["z"].detach().numpy()
    for k in ("rec", "kl_c", "kl_s", "c_loss"):
        if k in o:
            out[k] = float(o[k].detach())
    for k in ("mu_c", "logvar_c", "mu_s", "logvar_s"):
        out[k] = o[k].detach().numpy()
    out["xhat"] = o["xhat"].detach().numpy()
    out["grads"] = {k: g.detach().numpy() for k, g in o["grads"].items()}
    params = {k: v for k, v in P.items() if isinstance(v, torch.Tensor) and v.requires_grad}
    for k, p in params.items():
        p.grad = o["grads"][k].detach().clone()
    torch.optim.Adam(list(params.values()), lr=hp["lr"]).step()
    if mode == "mim":
        d = m["z"] // 2
        Mp = [v for v in M.values()]
        eopt = torch.optim.Adam(Mp, lr=hp["est_lr"])
        learn = []
        for j in range(5):
            a, b = fx["extra_noise"][j]
            with torch.no_grad():
                _, _, zz = R.vae_forward(P, X, torch.tensor(a, dtype=dtype), torch.tensor(b, dtype=dtype), arch, True)
            ll = R.learning_loss(M, zz[:, :d], zz[:, d:])
            eopt.zero_grad()
            ll.backward()
            eopt.step()
            learn.append(float(ll))
        out["mi_learning"] = np.array(learn)
        out["est_after"] = {k: v.detach().numpy() for k, v in M.items()}
    if mode == "tc":
        # factor step (trainer.py:680-699): a second train-mode forward with fresh noise on the updated VAE,
        # BCE of the discriminator on joint / factor-shuffled z, torch Adam on the discriminator
        a, b = fx["extra_noise"][0]
        with torch.no_grad():
            _, _, z2 = R.vae_forward(P, X, torch.tensor(a, dtype=dtype), torch.tensor(b, dtype=dtype), arch, True)
        Dp = list(D.values())
        for p_ in Dp:
            p_.grad = None
        fl = R.tc_factor_loss(D, z2.detach())
        fl.backward()
        out["z2"] = z2.numpy()
        out["factor_loss"] = float(fl.detach())
        out["disc_grad"] = {k: v.grad.detach().numpy().copy() for k, v in D.items()}
        torch.optim.Adam(Dp, lr=hp["factor_lr"]).step()
        out["disc_after"] = {k: v.detach().numpy() for k, v in D.items()}
    out["after"] = {k: p.detach().numpy() for k, p in params.items()}
    out["buffers"] = {k: v.detach().numpy() for k, v in P.items()
                      if k.endswith(("running_mean", "running_var", "num_batches_tracked"))}
    return out


def rel(a, b) -> float:
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-300))


def pick(fx: dict, prefix: str, name: str, full: np.ndarray) -> tuple:
    """(ours, golden) for a stored tensor: full for small ones, the stored sample for large ones."""
    flat = np.asarray(full).reshape(-1)
    idx = fx.get("gidx__" + name)
    return (flat if idx is None else flat[idx]), fx[prefix + name]
