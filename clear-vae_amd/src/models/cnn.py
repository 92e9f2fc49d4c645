"""Baseline CNN classifiers (reference code/src/models/cnn.py).  Comparison baselines, outside the
CLEAR-VAE hot path: plain PyTorch modules kept so the experiment scripts import."""

import torch.nn as nn


def _trunk(table, in_channel):
    layers = []
    c = in_channel
    for cout, k in table:
        layers += [nn.Conv2d(c, cout, k, 2, 1), nn.BatchNorm2d(cout), nn.ReLU()]
        c = cout
    return nn.Sequential(*layers, nn.Flatten())


class SimpleCNNClassifier(nn.Module):
    def __init__(self, n_class: int = 10, in_channel: int = 1) -> None:
        super().__init__()
        self.net = _trunk([(32, 3), (64, 3), (128, 3)], in_channel)
        self.cls_head = nn.Sequential(nn.Linear(2048, 256), nn.BatchNorm1d(256), nn.ReLU(), nn.Linear(256, n_class))

    def forward(self, x):
        return self.cls_head(self.net(x))


class SimpleCNN64Classifier(SimpleCNNClassifier):
    def __init__(self, n_class: int = 4, in_channel: int = 3) -> None:
        super().__init__(n_class, in_channel)
        self.net = _trunk([(32, 4), (64, 4), (128, 4), (256, 4), (512, 4)], in_channel)


class LAMCNNClassifier(SimpleCNNClassifier):
    def __init__(self, n_class: int = 10, in_channel: int = 1) -> None:
        super().__init__(n_class, in_channel)
        self.cls_head = nn.Linear(2048, n_class)


class LAMCNN64Classifier(SimpleCNN64Classifier):
    def __init__(self, n_class: int = 4, in_channel: int = 3) -> None:
        super().__init__(n_class, in_channel)
        self.cls_head = nn.Linear(2048, n_class)
