"""The drop-in surface on the CPU: the reference's module / function / class names
import from src.*, the model topology produces the reference's state_dict keys and shapes (the same
list oracle.cpu_ref.state_keys restates, which the golden generator loads strict=True into the real
reference modules), and the product path fails loudly instead of falling back to the CPU."""

import pytest
import torch


def test_reference_names_import():
    import src.losses as L
    import src.models.mi_estimator as MI
    import src.models.vae as V
    import src.trainer as T
    import src.utils.trainer_utils as U

    for n in ("VAE", "VAE64"):
        assert hasattr(V, n)
    for n in ("vae_loss", "contrastive_loss", "snn_loss", "logsumexp", "pairwise_cosine", "pairwise_l2",
              "pairwise_jeffrey_div", "pairwise_mahalanobis_dis", "pairwise_modified_l2_dis", "mutual_info_gap"):
        assert hasattr(L, n), n
    for n in ("CLUBSample", "L1OutUB"):
        assert hasattr(MI, n)
    for n in ("Trainer", "VAETrainer", "CLEARVAETrainer", "ClearMIMVAETrainer", "LogisticAnnealer",
              "DownstreamMLPTrainer", "SimpleCNNTrainer", "HierarchicalVAETrainer"):
        assert hasattr(T, n), n
    for n in ("get_clearvae_trainer", "get_clearmimvae_trainer", "get_cnn_trainer",
              "get_hierarchical_vae_trainer", "get_cleartcvae_trainer"):
        assert hasattr(U, n), n


@pytest.mark.parametrize("arch,z,c", [("VAE", 16, 1), ("VAE64", 64, 3), ("VAE", 10, 3)])
def test_state_dict_matches_reference_topology(arch, z, c):
    import src.models.vae as V
    from oracle import cpu_ref as R

    m = getattr(V, arch)(z, c)
    sd = m.state_dict()
    ref = R.state_keys(arch, z, c)
    assert list(sd.keys()) == [k for k, _ in ref]
    for k, shape in ref:
        assert tuple(sd[k].shape) == tuple(shape), k
    m.load_state_dict({k: torch.as_tensor(v) for k, v in R.det_state(arch, z, c).items()}, strict=True)
    assert m.z_dim == z // 2


def test_parameter_counts():
    import src.models.vae as V

    assert sum(p.numel() for p in V.VAE(16, 1).parameters()) == 290339
    assert sum(p.numel() for p in V.VAE64(64, 3).parameters()) == 5977545


def test_no_cpu_fallback():
    import src.models.vae as V

    m = V.VAE(16, 1)
    with pytest.raises(RuntimeError):
        m(torch.rand(4, 1, 28, 28))


def test_unknown_similarity_error():
    from src.losses import contrastive_loss

    mu = torch.zeros(4, 8)
    with pytest.raises(ValueError, match="unimplemented similarity measure."):
        contrastive_loss(mu, mu, torch.zeros(4, dtype=torch.long), "cityblock", 0.1)


def test_annealer_matches_reference_formula():
    import math

    from src.trainer import LogisticAnnealer

    a = LogisticAnnealer(loc=0, scale=1, beta=0.125)
    assert a.slope() == 0.125 / 2
    a.step()
    assert abs(a.slope() - 0.125 / (1 + math.exp(-1))) < 1e-15
