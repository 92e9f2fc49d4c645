"""Trainer factories with the reference's signatures (code/src/utils/trainer_utils.py).

The reference dispatches architecture / estimator names with ``eval``; here an explicit registry
accepts the same strings ("VAE", "VAE64", "CLUBSample", "L1OutUB", the CNN class names).
"""

import torch
import torch.nn as nn

from cvhip.plan import set_precision

from src.models.cnn import LAMCNN64Classifier, LAMCNNClassifier, SimpleCNN64Classifier, SimpleCNNClassifier
from src.models.mi_estimator import CLUB, CLUBMean, CLUBSample, InfoNCE, L1OutUB, VarUB
from src.models.vae import VAE, VAE64
from src.trainer import (
    ClearMIMVAETrainer,
    ClearTCVAETrainer,
    CLEARVAETrainer,
    HierarchicalVAETrainer,
    LAMCNNTrainer,
    SimpleCNNTrainer,
)

_REGISTRY = {
    c.__name__: c
    for c in (VAE, VAE64, SimpleCNNClassifier, SimpleCNN64Classifier, LAMCNNClassifier, LAMCNN64Classifier,
              CLUBSample, L1OutUB, CLUB, CLUBMean, VarUB, InfoNCE)
}


def _resolve(name):
    try:
        return _REGISTRY[name]
    except KeyError:
        raise NameError(f"name '{name}' is not defined") from None


def get_cnn_trainer(n_class, device, cnn_arch: str = "SimpleCNNClassifier", in_channel: int = 1,
                    verbose_period: int = 5):
    cnn = _resolve(cnn_arch)(n_class=n_class, in_channel=in_channel).to(device)
    optimizer = torch.optim.Adam(cnn.parameters(), lr=1e-4)
    return SimpleCNNTrainer(cnn, optimizer, torch.nn.CrossEntropyLoss(), verbose_period=verbose_period,
                            device=device)


def get_lamcnn_trainer(n_class, device, lam_coef, cnn_arch: str = "LAMCNNClassifier", in_channel: int = 1,
                       verbose_period: int = 5):
    cnn = _resolve(cnn_arch)(n_class=n_class, in_channel=in_channel).to(device)
    optimizer = torch.optim.Adam(cnn.parameters(), lr=1e-4)
    return LAMCNNTrainer(cnn, optimizer, torch.nn.CrossEntropyLoss(), {"lam_coef": lam_coef},
                         verbose_period=verbose_period, device=device)


def get_hierarchical_vae_trainer(beta, vae_lr, z_dim, group_mode, device, vae_arch: str = "VAE",
                                 in_channel: int = 1, verbose_period: int = 5):
    vae = _resolve(vae_arch)(total_z_dim=z_dim, in_channel=in_channel, group_mode=group_mode).to(device)
    optimizer = torch.optim.Adam(vae.parameters(), lr=vae_lr)
    return HierarchicalVAETrainer(vae, optimizer, hyperparameter={"beta": beta, "scale": 1, "loc": 0},
                                  verbose_period=verbose_period, device=device)


def get_clearvae_trainer(beta, ps, vae_lr, z_dim, alpha, temperature, device, vae_arch: str = "VAE",
                         in_channel: int = 1, verbose_period: int = 5, precision: str = "fp32"):
    """(trainer_utils.py:87-116).  `precision` (not in the reference, default its fp32): "bf16" runs the
    conv / linear contractions on bf16 MFMA operands (cvhip.plan.set_precision)."""
    vae = _resolve(vae_arch)(total_z_dim=z_dim, in_channel=in_channel).to(device)
    set_precision(vae, precision)
    optimizer = torch.optim.Adam(vae.parameters(), lr=vae_lr)
    return CLEARVAETrainer(
        vae, optimizer, sim_fn="cosine",
        hyperparameter={"temperature": temperature, "alpha": alpha, "beta": beta, "ps": ps, "loc": 0, "scale": 1},
        verbose_period=verbose_period, device=device,
    )


def get_cleartcvae_trainer(beta, la, vae_lr, factor_cls_lr, z_dim, alpha, temperature, device,
                           vae_arch: str = "VAE", in_channel: int = 1, verbose_period: int = 5,
                           precision: str = "fp32"):
    """(trainer_utils.py:119-157); `precision` as in get_clearvae_trainer."""
    vae = _resolve(vae_arch)(total_z_dim=z_dim, in_channel=in_channel).to(device)
    set_precision(vae, precision)
    factor_cls = nn.Sequential(nn.Linear(z_dim, z_dim), nn.ReLU(), nn.Linear(z_dim, 1), nn.Sigmoid()).to(device)
    vae_opt = torch.optim.Adam(vae.parameters(), lr=vae_lr)
    fac_opt = torch.optim.Adam(factor_cls.parameters(), lr=factor_cls_lr)
    return ClearTCVAETrainer(
        vae, factor_cls, optimizers={"vae_optim": vae_opt, "factor_optim": fac_opt}, sim_fn="cosine",
        hyperparameter={"temperature": temperature, "alpha": alpha, "beta": beta, "loc": 0, "scale": 1,
                        "lambda": la},
        verbose_period=verbose_period, device=device,
    )


def get_clearmimvae_trainer(beta, mi_estimator: str, la, vae_lr, mi_estimator_lr, z_dim, alpha, temperature,
                            device, vae_arch: str = "VAE", in_channel: int = 1, verbose_period: int = 5,
                            precision: str = "fp32"):
    """(trainer_utils.py:160-201); `precision` as in get_clearvae_trainer."""
    vae = _resolve(vae_arch)(total_z_dim=z_dim, in_channel=in_channel).to(device)
    set_precision(vae, precision)
    est = _resolve(mi_estimator)(x_dim=z_dim // 2, y_dim=z_dim // 2, hidden_size=z_dim).to(device)
    vae_opt = torch.optim.Adam(vae.parameters(), lr=vae_lr)
    est_opt = torch.optim.Adam(est.parameters(), lr=mi_estimator_lr)
    return ClearMIMVAETrainer(
        vae, est, optimizers={"vae_optim": vae_opt, "mi_estimator_optim": est_opt}, sim_fn="cosine",
        hyperparameter={"temperature": temperature, "beta": beta, "loc": 0, "scale": 1, "alpha": alpha,
                        "lambda": la},
        verbose_period=verbose_period, device=device,
    )
