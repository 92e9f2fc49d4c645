"""Batches above the one-workgroup caps (N > 4096) of the NT-Xent and CLUB-S / L1OutUB kernels: the reference
has no cap (losses.py:98-137, mi_estimator.py:108-198), so neither does the HIP path.

  * contrastive_loss (HIP autograd, src/losses.py) at N = 8192: the global-walk NT-Xent kernels with the row
    norms recomputed per pair (cv_latent.hip, NT_MAXBIG) against the oracle's blockwise restatement of the same
    row terms (oracle/cpu_ref.py contrastive_loss_blockwise, itself checked against the literal form at small N);
    loss and both gradients within 1e-4 relative (the north_star bar);
  * CLUBSample (injected permutation) and L1OutUB (closed form, oracle/cpu_ref.py l1out_closed) at N = 8192:
    the MI value and its gradients w.r.t. x, y and the estimator parameters within 1e-4;
  * the device permutation above 4096 (mi_perm_big_kernel: keyed Feistel bijection with cycle walking) is a
    bijection with a consistent inverse, differs call to call, and moves positions like a random permutation;
  * the fused CLEAR step at N = 8192 runs the big NT-Xent path inside its graph: its contrastive losses equal the
    blockwise oracle evaluated on the step's own heads."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N = 8192


def _rel(a, b):
    a, b = torch.as_tensor(a).double().reshape(-1).cpu(), torch.as_tensor(b).double().reshape(-1).cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("sim_fn,d,ps", [("cosine", 8, True), ("cosine", 8, False), ("jeffrey", 8, True),
                                         ("l2", 32, False)])
def test_contrastive_big_batch(sim_fn, d, ps):
    from oracle import cpu_ref as R
    from src.losses import contrastive_loss

    g = torch.Generator().manual_seed(8 + d)
    mu = torch.randn(N, d, generator=g, dtype=torch.float64)
    lv = 0.3 * torch.randn(N, d, generator=g, dtype=torch.float64)
    label = torch.randint(0, 10, (N,), generator=g)
    m_dev = mu.float().cuda().requires_grad_(True)
    l_dev = lv.float().cuda().requires_grad_(True)
    loss = contrastive_loss(m_dev, l_dev, label.cuda(), sim_fn, 0.1, ps=ps)
    loss.backward()
    torch.cuda.synchronize()
    m64, l64 = mu.clone().requires_grad_(True), lv.clone().requires_grad_(True)
    ref = R.contrastive_loss_blockwise(m64, l64, label, sim_fn, 0.1, ps)
    assert abs(float(loss) - float(ref)) <= 1e-4 * max(abs(float(ref)), 1e-3), (float(loss), float(ref))
    assert _rel(m_dev.grad, m64.grad) < 1e-4, _rel(m_dev.grad, m64.grad)
    if sim_fn not in ("cosine", "l2"):
        assert _rel(l_dev.grad, l64.grad) < 1e-4, _rel(l_dev.grad, l64.grad)


@pytest.mark.parametrize("kind", ["CLUBSample", "L1OutUB"])
def test_mi_big_batch(kind):
    from cvhip import rng
    from oracle import cpu_ref as R
    from src.models.mi_estimator import CLUBSample, L1OutUB

    d = 8
    g = torch.Generator().manual_seed(21)
    x = torch.randn(N, d, generator=g, dtype=torch.float64)
    y = torch.randn(N, d, generator=g, dtype=torch.float64)
    perm = torch.randperm(N, generator=g)
    md = R.det_mlp(d, 2 * d)
    est = (CLUBSample if kind == "CLUBSample" else L1OutUB)(d, d, 2 * d).cuda()
    est.load_state_dict({k: torch.tensor(v, dtype=torch.float32) for k, v in md.items()})
    rng.clear_injections()
    if kind == "CLUBSample":
        rng.inject_perm([perm])
    xd, yd = x.float().cuda().requires_grad_(True), y.float().cuda().requires_grad_(True)
    mi = est(xd, yd)
    mi.backward()
    torch.cuda.synchronize()
    M = R.to_torch(md)
    x64, y64 = x.clone().requires_grad_(True), y.clone().requires_grad_(True)
    ref = R.club_sample(M, x64, y64, perm) if kind == "CLUBSample" else R.l1out_closed(M, x64, y64)
    ref.backward()
    assert abs(float(mi) - float(ref)) <= 1e-4 * max(abs(float(ref)), 1.0), (float(mi), float(ref))
    assert _rel(xd.grad, x64.grad) < 1e-4 and _rel(yd.grad, y64.grad) < 1e-4, (_rel(xd.grad, x64.grad),
                                                                                _rel(yd.grad, y64.grad))
    for k, p in est.named_parameters():
        assert _rel(p.grad, M[k].grad) < 1e-4, (k, _rel(p.grad, M[k].grad))


@pytest.mark.parametrize("n", [N, 10000])
def test_clubsample_device_permutation_above_cap(n):
    """cv_mi_forward without an injected permutation at n > 4096: perm / invperm in the workspace (cv_mi.hip
    mi_work layout, as tests/test_gpu_rng.py reads them)."""
    from cvhip import _lib
    from cvhip.autograd import mlp_struct
    from src.models.mi_estimator import CLUBSample

    d = 8
    est = CLUBSample(d, d, 2 * d).cuda()
    x = torch.randn(n, d, device="cuda")
    y = torch.randn(n, d, device="cuda")
    work = torch.zeros(int(_lib.lib().cv_mi_workspace_bytes(n)) // 4 + 16, dtype=torch.float32, device="cuda")
    off = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = torch.empty((), device="cuda")
    nb, fp, gsz = 64, 2 + 128, 4 * 64 * 64 + 256
    base = (4 * 64 * 8 + nb * fp * 8 + nb * 8 + 64 + nb * gsz * 4) // 4
    perms = []
    for _ in range(3):
        _lib.call("cv_mi_forward", _lib.MI_CLUBSAMPLE, mlp_struct(est), x.data_ptr(), d, y.data_ptr(), d, n, None,
                  1234, off.data_ptr(), work.data_ptr(), out.data_ptr(), _lib.stream_handle())
        torch.cuda.synchronize()
        raw = work.view(torch.int32).cpu().numpy()
        perm, inv = raw[base: base + n].copy(), raw[base + n: base + 2 * n].copy()
        assert np.array_equal(np.sort(perm), np.arange(n)), "not a permutation"
        assert np.array_equal(inv[perm], np.arange(n)), "inverse inconsistent"
        assert np.isfinite(float(out))
        perms.append(perm)
    assert int(off.item()) == 3  # one offset step per call
    for a, b in zip(perms, perms[1:]):
        assert not np.array_equal(a, b), "same permutation on consecutive calls"
    fixed = sum(int((p == np.arange(n)).sum()) for p in perms)
    assert fixed < 20, fixed
    assert np.mean([np.abs(p - np.arange(n)).mean() for p in perms]) > n / 4


def test_fused_clear_step_big_batch():
    """The fused CLEAR step (VAE, z = 16) at N = 8192: the contrastive losses it reports are the blockwise oracle's
    on the step's own heads (mu_c / mu_s of ws.heads), i.e. the big NT-Xent kernels run inside the step."""
    from cvhip.engine import ClearStep
    from oracle import cpu_ref as R
    from src.utils.trainer_utils import get_clearvae_trainer

    torch.manual_seed(0)
    tr = get_clearvae_trainer(beta=1 / 8, ps=True, vae_lr=5e-4, z_dim=16, alpha=100, temperature=0.1, device="cuda")
    eng = ClearStep.build(tr, "clear")
    assert eng is not None
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.rand(N, 1, 28, 28, generator=g, device="cuda")
    L = torch.randint(0, 10, (N,), generator=g, device="cuda")
    losses = eng.step(X, L).cpu()
    torch.cuda.synchronize()
    assert torch.isfinite(losses[:5]).all()
    h = eng.last_workspace(N).heads.double().cpu()
    d = 8
    lab = L.cpu()
    with torch.no_grad():
        c = R.contrastive_loss_blockwise(h[:, :d], h[:, d:2 * d], lab, "cosine", 0.1, False)
        s = R.contrastive_loss_blockwise(h[:, 2 * d:3 * d], h[:, 3 * d:], lab, "cosine", 0.1, True)
    assert abs(float(losses[3]) - float(c)) <= 1e-4 * abs(float(c)), (float(losses[3]), float(c))
    assert abs(float(losses[4]) - float(s)) <= 1e-4 * abs(float(s)), (float(losses[4]), float(s))
