"""Trainers with the reference's classes, constructor signatures, hyperparameter keys, step order,
printed values and return values (code/src/trainer.py).

CLEARVAETrainer / ClearMIMVAETrainer (the hot path) run each training step
as one fused HIP program (cvhip.engine.ClearStep: forward, ELBO, contrastive / MI terms, backward,
BatchNorm bookkeeping and Adam on a flat parameter arena, replayed as a HIP graph).  When the caller's
setup is outside what the fused step supports (e.g. an optimizer that is not a single-group Adam
over all VAE parameters), they fall back to the module-level HIP path (cvhip.autograd), which
replays the reference's loop literally.  Neither path computes on the CPU.

Per-step scalars that the reference reads with float() every step (trainer.py:486-492, 859, 888)
are kept on the device and copied once per epoch when the progress bar is disabled.
ClearTCVAETrainer runs fused too (mode "tc": the factor discriminator's density-ratio
term and its BCE step as HIP kernels), and so does HierarchicalVAETrainer (mode "group":
the GVAE / ML-VAE group evidence as label-segmented device reductions).  The remaining trainers (CNN
baselines, downstream probe) are outside the hot path and keep the reference's
PyTorch loops.
"""

from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.optim.optimizer import Optimizer
from torch.utils.data import DataLoader
from tqdm import tqdm

from src.losses import accurary, auc, contrastive_loss, lam_loss, mutual_info_gap, vae_loss
from src.models.vae import VAE


class LogisticAnnealer:
    """beta / (1 + exp(-(t - loc)/scale)) with t = optimizer steps taken (trainer.py:22-38)."""

    def __init__(self, loc, scale, beta) -> None:
        self.current_step = 0
        self.loc = loc
        self.scale = scale
        self.beta = beta

    def __call__(self, kl_loss) -> torch.Tensor:
        return kl_loss * self.slope()

    def slope(self) -> float:
        exponent = -(self.current_step - self.loc) / self.scale
        return self.beta / (1 + math.exp(exponent))

    def step(self) -> None:
        self.current_step += 1


class Trainer:
    def __init__(self, model: nn.Module, optimizer: Optimizer, verbose_period: int, device: torch.device,
                 transform=None) -> None:
        self.model = model
        self.optimizer = optimizer
        self.verbose_period = verbose_period
        self.device = device
        self.transform = transform

    def fit(self, epochs: int, train_loader: DataLoader, valid_loader: None | DataLoader = None):
        for epoch in range(epochs):
            verbose = (epoch % self.verbose_period) == 0
            self._train(train_loader, verbose, epoch)
            if valid_loader is not None:
                self._valid(valid_loader, verbose, epoch)

    def evaluate(self, **kwarg):
        pass

    def _train(self, **kwarg):
        pass

    def _valid(self, **kwarg):
        pass


class VAETrainer(Trainer):
    def _valid(self, dataloader, verbose, epoch_id):
        if verbose:
            mig, mse = self.evaluate(dataloader, verbose, epoch_id)
            print(f"gMIG: {round(mig, 3)}; mse: {round(float(mse), 3)}")


def _batch(batch, device, transform):
    X, label = batch[0], batch[1].reshape(-1).long()
    X, label = X.to(device), label.to(device)
    if transform:
        X = transform(X)
    return X, label


# ----------------------------------------------------------------------------- CLEAR-VAE


class _ClearEval:
    """evaluate() shared by the CLEAR trainers (trainer.py:495-570, 899-965): eval-mode forward on the
    HIP path under no_grad, the same losses, gMIG on the CPU."""

    def _evaluate(self, dataloader, verbose, epoch_id, last_name, last_fn):
        vae = self.model
        vae.eval()
        hp = self.hyperparameter
        totals = [0.0] * 5
        labels, lat_c, lat_s = [], [], []
        with torch.no_grad():
            for batch in tqdm(dataloader, disable=not verbose, desc=f"val-epoch {epoch_id}"):
                X, label = _batch(batch, self.device, self.transform)
                X_hat, lp, z = vae(X, explicit=True)
                rec, kl_c, kl_s = vae_loss(X_hat, X, **lp)
                c_loss = contrastive_loss(mu=lp["mu_c"], logvar=lp["logvar_c"], label=label, sim_fn=self.sim_fn,
                                          temperature=hp["temperature"])
                last = last_fn(lp, label, z)
                for i, v in enumerate((rec, kl_c, kl_s, c_loss, last)):
                    totals[i] += v
                labels.append(label)
                lat_c.append(z[:, : vae.z_dim])
                lat_s.append(z[:, vae.z_dim:])
        mig = mutual_info_gap(torch.cat(labels), torch.cat(lat_c), torch.cat(lat_s))
        nb = len(dataloader)
        mse = float(totals[0] / nb)
        if verbose:
            print(
                ("val_recontr_loss={:.3f}, val_kl_c={:.3f}, val_kl_s={:.3f}, val_c_loss={:.3f}, val_" + last_name
                 + "={:.3f}").format(*[t / nb for t in totals])
            )
        return mig, mse


class CLEARVAETrainer(VAETrainer, _ClearEval):
    def __init__(self, model: VAE, optimizer: Optimizer, sim_fn: str, hyperparameter: dict[str, float],
                 verbose_period: int, device: torch.device, transform=None) -> None:
        super().__init__(model, optimizer, verbose_period, device, transform)
        self.sim_fn = sim_fn
        self.hyperparameter = hyperparameter
        self.annealer = LogisticAnnealer(loc=hyperparameter["loc"], scale=hyperparameter["scale"],
                                         beta=hyperparameter["beta"])
        self._engine = None
        self.use_fused = True

    def _fused(self):
        if not self.use_fused:
            return None
        from cvhip.engine import ClearStep

        if self._engine is None or not self._engine.compatible():
            self._engine = ClearStep.build(self, mode="clear")
        return self._engine

    def _train(self, dataloader: DataLoader, verbose: bool, epoch_id: int):
        vae = self.model
        vae.train()
        hp = self.hyperparameter
        engine = self._fused()
        with tqdm(dataloader, unit="batch", mininterval=0, disable=not verbose) as bar:
            bar.set_description(f"Epoch {epoch_id}")
            for batch in bar:
                X, label = _batch(batch, self.device, self.transform)
                if engine is not None and engine.accepts(X):
                    if getattr(self, "_resync", False):
                        engine.resync_from_host()
                        self._resync = False
                    losses = engine.step(X, label)
                    self.annealer.step()
                    if verbose:
                        v = losses.tolist()
                        s_loss = v[4] if hp["ps"] else -v[4]
                        bar.set_postfix(recontr_loss=v[0], kl_c=v[1], kl_s=v[2], c_loss=v[3], s_loss=s_loss)
                    continue
                if engine is not None:
                    engine.sync_host_state()
                    self._resync = True
                self.optimizer.zero_grad()
                X_hat, lp = vae(X)
                rec, kl_c, kl_s = vae_loss(X_hat, X, **lp)
                c_loss = contrastive_loss(mu=lp["mu_c"], logvar=lp["logvar_c"], label=label, sim_fn=self.sim_fn,
                                          temperature=hp["temperature"])
                s_loss = contrastive_loss(mu=lp["mu_s"], logvar=lp["logvar_s"], label=label, sim_fn=self.sim_fn,
                                          temperature=hp["temperature"], ps=hp["ps"])
                if not hp["ps"]:
                    s_loss = -s_loss
                loss = (rec + self.annealer(kl_c) + self.annealer(kl_s) + hp["alpha"] * c_loss
                        + hp["alpha"] * s_loss)
                loss.backward()
                self.optimizer.step()
                self.annealer.step()
                if verbose:
                    bar.set_postfix(recontr_loss=float(rec), kl_c=float(kl_c), kl_s=float(kl_s),
                                    c_loss=float(c_loss), s_loss=float(s_loss))
        if engine is not None:
            engine.sync_host_state()

    def evaluate(self, dataloader, verbose, epoch_id):
        hp = self.hyperparameter

        def s_term(lp, label, z):
            s = contrastive_loss(mu=lp["mu_s"], logvar=lp["logvar_s"], label=label, sim_fn=self.sim_fn,
                                 temperature=hp["temperature"], ps=hp["ps"])
            return s if hp["ps"] else -s

        return self._evaluate(dataloader, verbose, epoch_id, "s_loss", s_term)


# ----------------------------------------------------------------------------- CLEAR-MIM


class ClearMIMVAETrainer(VAETrainer, _ClearEval):
    def __init__(self, model: VAE, mi_estimator: nn.Module, optimizers: dict[str, Optimizer], sim_fn: str,
                 hyperparameter: dict[str, float], verbose_period: int, device: torch.device,
                 transform=None) -> None:
        super().__init__(model, optimizers["vae_optim"], verbose_period, device, transform)
        self.sim_fn = sim_fn
        self.mi_estimator_optimizer = optimizers["mi_estimator_optim"]
        self.mi_estimator = mi_estimator
        self.hyperparameter = hyperparameter
        self.annealer = LogisticAnnealer(loc=hyperparameter["loc"], scale=hyperparameter["scale"],
                                         beta=hyperparameter["beta"])
        self._engine = None
        self.use_fused = True

    def _fused(self):
        if not self.use_fused:
            return None
        from cvhip.engine import ClearStep

        if self._engine is None or not self._engine.compatible():
            self._engine = ClearStep.build(self, mode="mim")
        return self._engine

    def fit(self, epochs: int, train_loader: DataLoader, valid_loader: None | DataLoader = None):
        mi_losses, mi_learning_losses = [], []
        for epoch in range(epochs):
            verbose = (epoch % self.verbose_period) == 0
            self._train(train_loader, verbose, epoch, mi_losses, mi_learning_losses)
            if valid_loader is not None:
                self._valid(valid_loader, verbose, epoch)
        return mi_losses, mi_learning_losses

    def _train(self, dataloader: DataLoader, verbose: bool, epoch_id: int, mi_losses: list,
               mi_learning_losses: list):
        vae, est = self.model, self.mi_estimator
        vae.train()
        est.train()
        hp = self.hyperparameter
        engine = self._fused()
        dev_log = []  # device-side per-step scalars, converted once at the end of the epoch
        with tqdm(dataloader, unit="batch", mininterval=0, disable=not verbose) as bar:
            bar.set_description(f"Epoch {epoch_id}")
            for batch in bar:
                X, label = _batch(batch, self.device, self.transform)
                if engine is not None and engine.accepts(X):
                    if getattr(self, "_resync", False):
                        engine.resync_from_host()
                        self._resync = False
                    losses, learn = engine.step(X, label)
                    self.annealer.step()
                    dev_log.append((losses[5:6].clone(), learn))
                    if verbose:
                        v = losses.tolist()
                        bar.set_postfix(recontr_loss=v[0], kl_c=v[1], kl_s=v[2], c_loss=v[3], mi_loss=v[5])
                    continue
                if engine is not None:
                    engine.sync_host_state()
                    self._resync = True
                X_hat, lp, z = vae(X, explicit=True)
                self.optimizer.zero_grad()
                rec, kl_c, kl_s = vae_loss(X_hat, X, **lp)
                c_loss = contrastive_loss(mu=lp["mu_c"], logvar=lp["logvar_c"], label=label, sim_fn=self.sim_fn,
                                          temperature=hp["temperature"])
                mi = est(z[:, : vae.z_dim], z[:, vae.z_dim:])
                loss = (rec + self.annealer(kl_c) + self.annealer(kl_s) + hp["alpha"] * c_loss
                        + hp["lambda"] * mi)
                loss.backward()
                self.optimizer.step()
                self.annealer.step()
                learn = []
                for _ in range(5):
                    _, _, z2 = vae(X, explicit=True)
                    z2 = z2.detach()
                    ll = est.learning_loss(z2[:, : vae.z_dim], z2[:, vae.z_dim:])
                    self.mi_estimator_optimizer.zero_grad()
                    ll.backward()
                    self.mi_estimator_optimizer.step()
                    learn.append(ll.detach().reshape(1))
                dev_log.append((mi.detach().reshape(1), torch.cat(learn)))
                if verbose:
                    bar.set_postfix(recontr_loss=float(rec), kl_c=float(kl_c), kl_s=float(kl_s),
                                    c_loss=float(c_loss), mi_loss=float(mi))
        if engine is not None:
            engine.sync_host_state()
        if dev_log:
            mis = torch.cat([m for m, _ in dev_log]).tolist()
            lls = torch.cat([ll for _, ll in dev_log]).tolist()
            mi_losses.extend(mis)
            mi_learning_losses.extend(lls)

    def evaluate(self, dataloader, verbose, epoch_id):
        est = self.mi_estimator
        est.eval()

        def mi_term(lp, label, z):
            return est(z[:, : self.model.z_dim], z[:, self.model.z_dim:])

        return self._evaluate(dataloader, verbose, epoch_id, "mi_loss", mi_term)


# ----------------------------------------------------------------------------- outside the hot path


class DownstreamMLPTrainer(Trainer):
    """MLP probe on mu_c of a frozen VAE (trainer.py:95-165); vae.encode runs on the HIP path."""

    def __init__(self, vae: nn.Module, model: nn.Module, optimizer: Optimizer, criterion: nn.Module,
                 verbose_period: int, device: torch.device, transform=None) -> None:
        super().__init__(model, optimizer, verbose_period, device, transform)
        self.criterion = criterion
        self.vae = vae

    def _train(self, dataloader: DataLoader, verbose: bool, epoch_id: int):
        self.model.train()
        with tqdm(dataloader, unit="batch", disable=not verbose) as bar:
            bar.set_description(f"epoch {epoch_id}")
            for batch in bar:
                X, y = batch[0], batch[1].reshape(-1).long()
                X, y = X.to(self.device), y.to(self.device)
                if self.transform:
                    X = self.transform(X)
                self.optimizer.zero_grad()
                logits = self.model(self.vae.encode(X)[0])
                loss = self.criterion(logits, y)
                loss.backward()
                self.optimizer.step()
                if verbose:
                    bar.set_postfix(loss=float(loss))

    def _valid(self, dataloader: DataLoader, verbose: bool, epoch_id: int):
        if verbose:
            (aupr, auroc), acc = self.evaluate(dataloader, verbose, epoch_id)
            print("val_aupr:", aupr)
            print(np.mean(list(aupr.values())).round(3))
            print("val_auroc:", auroc)
            print(np.mean(list(auroc.values())).round(3))
            print("val_acc:", acc.numpy().round(3))

    def evaluate(self, dataloader: DataLoader, verbose: bool, epoch_id: int):
        self.model.eval()
        ys, logits = [], []
        with torch.no_grad():
            for batch in tqdm(dataloader, disable=not verbose, desc=f"val-epoch {epoch_id}"):
                X, y = batch[0], batch[1].reshape(-1)
                logits.append(self.model(self.vae.encode(X.to(self.device))[0]))
                ys.append(y)
        ys, logits = torch.cat(ys), torch.cat(logits)
        return auc(logits, ys), accurary(logits, ys)


class SimpleCNNTrainer(Trainer):
    def __init__(self, model: nn.Module, optimizer: Optimizer, criterion: nn.Module, verbose_period: int,
                 device: torch.device, transform=None) -> None:
        super().__init__(model, optimizer, verbose_period, device, transform)
        self.criterion = criterion

    def _train(self, dataloader: DataLoader, verbose: bool, epoch_id: int):
        self.model.train()
        with tqdm(dataloader, unit="batch", disable=not verbose) as bar:
            bar.set_description(f"epoch {epoch_id}")
            for batch in bar:
                X, y = _batch(batch, self.device, self.transform)
                self.optimizer.zero_grad()
                loss = self.criterion(self.model(X), y)
                loss.backward()
                self.optimizer.step()
                if verbose:
                    bar.set_postfix(loss=float(loss))

    def _valid(self, dataloader: DataLoader, verbose: bool, epoch_id: int):
        if verbose:
            (aupr, auroc), acc = self.evaluate(dataloader, verbose, epoch_id)
            print("val_aupr:", aupr)
            print(np.mean(list(aupr.values())).round(3))
            print("val_auroc:", auroc)
            print(np.mean(list(auroc.values())).round(3))
            print("val_acc:", acc.numpy().round(3))

    def evaluate(self, dataloader: DataLoader, verbose: bool, epoch_id: int):
        self.model.eval()
        ys, logits = [], []
        with torch.no_grad():
            for batch in tqdm(dataloader, disable=not verbose, desc=f"val-epoch {epoch_id}"):
                X, y = batch[0], batch[1].reshape(-1)
                logits.append(self.model(X.to(self.device)))
                ys.append(y)
        ys, logits = torch.cat(ys), torch.cat(logits)
        return auc(logits, ys), accurary(logits, ys)


class LAMCNNTrainer(SimpleCNNTrainer):
    def __init__(self, model: nn.Module, optimizer: Optimizer, criterion: nn.Module, hyperparameter: dict,
                 verbose_period: int, device: torch.device, transform=None) -> None:
        super().__init__(model, optimizer, criterion, verbose_period, device, transform)
        self.hyperparameter = hyperparameter

    def ss_pairing(self, x, y):
        """Stratified shuffle: every sample is paired with a random sample of the same label
        (trainer.py:249-257)."""
        new_x = x.clone()
        for c in torch.unique(y):
            idx = (y == c).nonzero(as_tuple=True)[0]
            perm = torch.randperm(idx.shape[0])
            new_x[idx] = x[idx[perm.to(idx.device)]]
        return new_x

    def _train(self, dataloader: DataLoader, verbose: bool, epoch_id: int):
        """(X, y) batches, as the reference's callers pass them (trainer.py:259-288)."""
        cnn = self.model
        cnn.train()
        lam_coef = self.hyperparameter["lam_coef"]
        with tqdm(dataloader, unit="batch", disable=not verbose) as bar:
            bar.set_description(f"epoch {epoch_id}")
            for batch in bar:
                X, y = _batch(batch, self.device, self.transform)
                X_tilde = self.ss_pairing(X, y)
                self.optimizer.zero_grad()
                loss_ce = self.criterion(cnn(X), y)
                loss_lam = lam_loss(cnn.net(X), cnn.net(X_tilde), y, cnn.cls_head.weight)
                loss = loss_ce + lam_coef * loss_lam
                loss.backward()
                self.optimizer.step()
                bar.set_postfix(ce_loss=float(loss_ce), lam_loss=float(loss_lam))


class HierarchicalVAETrainer(VAETrainer):
    """GVAE / ML-VAE baselines (trainer.py:291-412).  Each step runs as one fused HIP program
    (cvhip.engine.ClearStep, mode "group"): the group evidence of vae.py:159-223 segmented by label on the
    device (cv_group_forward / cv_group_backward), kl_c over the groups and the B/m adjustment of rec and
    kl_s (trainer.py:322-324, 344-349) folded into the backward seed and the latent kernel.  Setups outside
    the fused contract run the reference's loop on the module-level HIP path."""

    def __init__(self, model: VAE, optimizer: Optimizer, hyperparameter: dict[str, float], verbose_period: int,
                 device: torch.device, transform=None) -> None:
        super().__init__(model, optimizer, verbose_period, device, transform)
        self.hyperparameter = hyperparameter
        self.annealer = LogisticAnnealer(loc=hyperparameter["loc"], scale=hyperparameter["scale"],
                                         beta=hyperparameter["beta"])
        self._engine = None
        self.use_fused = True

    def _fused(self):
        if not self.use_fused:
            return None
        from cvhip.engine import ClearStep

        if self._engine is None or not self._engine.compatible():
            self._engine = ClearStep.build(self, mode="group")
        return self._engine

    def fit(self, epochs: int, train_loader: DataLoader, valid_loader: None | DataLoader = None,
            eval_evidence_acc: bool = False):
        for epoch in range(epochs):
            verbose = (epoch % self.verbose_period) == 0
            self._train(train_loader, verbose, epoch)
            if valid_loader is not None:
                self._valid(valid_loader, verbose, epoch, eval_evidence_acc)

    def _group_adjust(self, B, m, *losses):
        return [loss * B / m for loss in losses]

    def _train(self, dataloader: DataLoader, verbose: bool, epoch_id: int):
        vae = self.model
        vae.train()
        engine = self._fused()
        with tqdm(dataloader, unit="batch", mininterval=0, disable=not verbose) as bar:
            bar.set_description(f"epoch {epoch_id}")
            for batch in bar:
                X, label = _batch(batch, self.device, None)
                if engine is not None and engine.accepts(X):
                    if getattr(self, "_resync", False):
                        engine.resync_from_host()
                        self._resync = False
                    losses = engine.step(X, label)
                    self.annealer.step()
                    if verbose:
                        v = losses.tolist()
                        bar.set_postfix(reconstr_loss=v[0], kl_c=v[1], kl_s=v[2])
                    continue
                if engine is not None:
                    engine.sync_host_state()
                    self._resync = True
                B, m = X.size(0), len(label.unique())
                if self.transform:
                    X = self.transform(X)
                self.optimizer.zero_grad()
                X_hat, lp = vae(X, label=label)
                rec, kl_c, kl_s = vae_loss(X_hat, X, **lp)
                rec, kl_s = self._group_adjust(B, m, rec, kl_s)
                loss = rec + self.annealer(kl_c) + self.annealer(kl_s)
                loss.backward()
                self.optimizer.step()
                self.annealer.step()
                if verbose:
                    bar.set_postfix(reconstr_loss=float(rec), kl_c=float(kl_c), kl_s=float(kl_s))
        if engine is not None:
            engine.sync_host_state()

    def _valid(self, dataloader, verbose, epoch_id, with_evidence_acc=False):
        if verbose:
            mig, mse = self.evaluate(dataloader, verbose, epoch_id, with_evidence_acc)
            print(f"gMIG: {round(mig, 3)}; mse: {round(float(mse), 3)}")

    def evaluate(self, dataloader, verbose, epoch_id, with_evidence_acc=False):
        vae = self.model
        vae.eval()
        tot = [0.0, 0.0, 0.0]
        labels, lat_c, lat_s = [], [], []
        with torch.no_grad():
            for batch in tqdm(dataloader, disable=not verbose, desc=f"val-epoch {epoch_id}"):
                X, label = _batch(batch, self.device, None)
                if with_evidence_acc:
                    X_hat, lp, z = vae(X, label, explicit=True)
                else:
                    X_hat, lp, z = vae(X, explicit=True)
                for i, v in enumerate(vae_loss(X_hat, X, **lp)):
                    tot[i] += v
                labels.append(label)
                lat_c.append(z[:, : vae.z_dim])
                lat_s.append(z[:, vae.z_dim:])
        mig = mutual_info_gap(torch.cat(labels), torch.cat(lat_c), torch.cat(lat_s))
        nb = len(dataloader)
        mse = float(tot[0] / nb)
        if verbose:
            print("val_recontr_loss={:.3f}, val_kl_c={:.3f}, val_kl_s={:.3f}".format(*[t / nb for t in tot]))
        return mig, mse


def factor_shuffling(z: torch.Tensor, strategy: str = "permute_1"):
    """(trainer.py:573-587)"""
    d = int(z.shape[1] / 2)
    z_c, z_s = z[:, :d], z[:, d:]
    if strategy == "full":
        return torch.cat([z_c, z_s[torch.randperm(z_s.shape[0])]], dim=1)
    if strategy == "permute_1":
        return torch.cat([z_c, torch.cat([z_s[1:, :], z_s[0, :][None]], dim=0)], dim=1)
    raise ValueError("this strategy is not implemented yet")


class ClearTCVAETrainer(VAETrainer, _ClearEval):
    """CLEAR-TC (trainer.py:590-778).  Each step runs as one fused HIP program (cvhip.engine.ClearStep,
    mode "tc"): the VAE step with the factor discriminator's density-ratio term relu(log(D/(1-D))).mean()
    (cv_tc_forward), a second train-mode forward with fresh noise, and the discriminator's BCE step on
    joint vs factor-shuffled z (cv_tc_learning_step + Adam).  Setups outside the fused contract (another
    discriminator architecture or optimizer) run the reference's loop with the VAE on the autograd HIP
    path and the discriminator in PyTorch."""

    def __init__(self, model: VAE, factor_cls: nn.Module, optimizers: dict[str, Optimizer], sim_fn: str,
                 hyperparameter: dict[str, float], verbose_period: int, device: torch.device,
                 transform=None) -> None:
        super().__init__(model, optimizers["vae_optim"], verbose_period, device, transform)
        self.sim_fn = sim_fn
        self.factor_optimizer = optimizers["factor_optim"]
        self.factor_cls = factor_cls
        self.hyperparameter = hyperparameter
        self.annealer = LogisticAnnealer(loc=hyperparameter["loc"], scale=hyperparameter["scale"],
                                         beta=hyperparameter["beta"])
        self._engine = None
        self.use_fused = True

    def _fused(self):
        if not self.use_fused:
            return None
        from cvhip.engine import ClearStep

        if self._engine is None or not self._engine.compatible():
            self._engine = ClearStep.build(self, mode="tc")
        return self._engine

    def fit(self, epochs: int, train_loader: DataLoader, valid_loader: None | DataLoader = None):
        factor_d_losses = []
        for epoch in range(epochs):
            verbose = (epoch % self.verbose_period) == 0
            self._train(train_loader, verbose, epoch, factor_d_losses)
            if valid_loader is not None:
                self._valid(valid_loader, verbose, epoch)
        return factor_d_losses

    def _train(self, dataloader: DataLoader, verbose: bool, epoch_id: int, factor_d_losses: list):
        vae, cls = self.model, self.factor_cls
        vae.train()
        cls.train()
        hp = self.hyperparameter
        engine = self._fused()
        log = []
        with tqdm(dataloader, unit="batch", mininterval=0, disable=not verbose) as bar:
            bar.set_description(f"Epoch {epoch_id}")
            for batch in bar:
                X, label = _batch(batch, self.device, self.transform)
                if engine is not None and engine.accepts(X):
                    if getattr(self, "_resync", False):
                        engine.resync_from_host()
                        self._resync = False
                    losses, fl = engine.step(X, label)
                    self.annealer.step()
                    log.append(fl)
                    if verbose:
                        v = losses.tolist()
                        bar.set_postfix(factor_cls_loss=float(fl), recontr_loss=v[0], kl_c=v[1], kl_s=v[2],
                                        c_loss=v[3], mi_loss=v[5])
                    continue
                if engine is not None:
                    engine.sync_host_state()
                    self._resync = True
                X_hat, lp, z = vae(X, explicit=True)
                self.optimizer.zero_grad()
                rec, kl_c, kl_s = vae_loss(X_hat, X, **lp)
                c_loss = contrastive_loss(mu=lp["mu_c"], logvar=lp["logvar_c"], label=label, sim_fn=self.sim_fn,
                                          temperature=hp["temperature"])
                d_score = cls(z)
                mi_loss = F.relu(torch.log(d_score / (1 - d_score))).mean()
                loss = (rec + self.annealer(kl_c) + self.annealer(kl_s) + hp["alpha"] * c_loss
                        + hp["lambda"] * mi_loss)
                loss.backward()
                self.optimizer.step()
                self.annealer.step()
                _, _, z = vae(X, explicit=True)
                z = z.detach()
                self.factor_optimizer.zero_grad()
                dj = cls(z)
                dm = cls(factor_shuffling(z))
                factor_loss = nn.BCELoss()(torch.cat([dj, dm], dim=0),
                                           torch.cat([torch.ones_like(dj), torch.zeros_like(dm)], dim=0))
                log.append(factor_loss.detach().reshape(1))
                factor_loss.backward()
                self.factor_optimizer.step()
                if verbose:
                    bar.set_postfix(factor_cls_loss=float(factor_loss), recontr_loss=float(rec), kl_c=float(kl_c),
                                    kl_s=float(kl_s), c_loss=float(c_loss), mi_loss=float(mi_loss))
        if engine is not None:
            engine.sync_host_state()
        if log:
            factor_d_losses.extend(torch.cat([t.reshape(1) for t in log]).tolist())

    def evaluate(self, dataloader, verbose, epoch_id):
        self.factor_cls.eval()

        def mi_term(lp, label, z):
            d = self.factor_cls(z)
            return F.relu(torch.log(d / (1 - d))).mean()

        return self._evaluate(dataloader, verbose, epoch_id, "mi_loss", mi_term)
