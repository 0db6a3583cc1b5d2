"""Vertical-FL party models (reference: `model/finance/*.py`, `classical_vertical_fl/party_models.py`)."""
import torch
import torch.nn as nn


class LocalModel(nn.Module):
    """Host/guest feature extractor: Linear → LeakyReLU."""

    def __init__(self, input_dim, output_dim):
        super().__init__()
        self.input_dim, self.output_dim = input_dim, output_dim
        self.classifier = nn.Sequential(nn.Linear(input_dim, output_dim), nn.LeakyReLU())

    def forward(self, x):
        return self.classifier(x)


class DenseModel(nn.Module):
    """Party-local linear head producing partial logits (summed across parties)."""

    def __init__(self, input_dim, output_dim, bias=True):
        super().__init__()
        self.classifier = nn.Linear(input_dim, output_dim, bias=bias)

    def forward(self, x):
        return self.classifier(x)


class VFLClassifier(nn.Module):
    def __init__(self, input_dim, output_dim):
        super().__init__()
        self.fc = nn.Linear(input_dim, output_dim)

    def forward(self, x):
        return self.fc(x)


class VFLFeatureExtractor(nn.Module):
    def __init__(self, input_dim, output_dim):
        super().__init__()
        self.fc = nn.Sequential(nn.Linear(input_dim, output_dim), nn.ReLU())

    def forward(self, x):
        return self.fc(x)
