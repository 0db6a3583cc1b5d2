"""Synthetic federated datasets with the shapes of the reference's datasets.

There is no network in this environment (and the north star asks for synthetic
data), so every dataset the reference knows (`data/data_loader.py:29-325`) has a
synthetic twin with the same tensor shapes / class counts. Samples are drawn
from class-conditional distributions so models actually learn (needed for the
FedAvg ≡ centralized and convergence checks):

* images  : x = 0.5·μ_y + 0.5·N(0,1), μ_y a smooth per-class pattern
* vectors : x = μ_y + N(0, σ²) (LR-style)
* tokens  : per-class unigram distributions over the vocabulary
"""
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np
import torch


@dataclass(frozen=True)
class DatasetSpec:
    name: str
    kind: str               # "image" | "vector" | "tokens" | "nwp" | "multilabel"
    shape: Tuple[int, ...]  # per-sample input shape
    num_classes: int
    train_size: int         # reference default train set size (synthetic uses a per-client count)
    test_size: int
    vocab: int = 0


SPECS: Dict[str, DatasetSpec] = {
    "mnist": DatasetSpec("mnist", "vector", (784,), 10, 60000, 10000),
    "femnist": DatasetSpec("femnist", "image", (1, 28, 28), 62, 671585, 77483),
    "fed_emnist": DatasetSpec("fed_emnist", "image", (1, 28, 28), 62, 671585, 77483),
    "synthetic_1_1": DatasetSpec("synthetic_1_1", "vector", (60,), 10, 20000, 2000),
    "cifar10": DatasetSpec("cifar10", "image", (3, 32, 32), 10, 50000, 10000),
    "cifar100": DatasetSpec("cifar100", "image", (3, 32, 32), 100, 50000, 10000),
    "fed_cifar100": DatasetSpec("fed_cifar100", "image", (3, 24, 24), 100, 50000, 10000),
    "cinic10": DatasetSpec("cinic10", "image", (3, 32, 32), 10, 90000, 90000),
    "ILSVRC2012": DatasetSpec("ILSVRC2012", "image", (3, 224, 224), 1000, 1281167, 50000),
    "gld23k": DatasetSpec("gld23k", "image", (3, 224, 224), 203, 23080, 1959),
    "gld160k": DatasetSpec("gld160k", "image", (3, 224, 224), 2028, 164172, 19526),
    "shakespeare": DatasetSpec("shakespeare", "nwp", (80,), 90, 413629, 103180, vocab=90),
    "fed_shakespeare": DatasetSpec("fed_shakespeare", "nwp", (80,), 90, 16068, 2356, vocab=90),
    "stackoverflow_nwp": DatasetSpec("stackoverflow_nwp", "nwp", (20,), 10004, 135818730, 16586035, vocab=10004),
    "stackoverflow_lr": DatasetSpec("stackoverflow_lr", "multilabel", (10000,), 500, 135818730, 16586035),
    "text_cls": DatasetSpec("text_cls", "tokens", (128,), 4, 120000, 7600, vocab=30522),
    "agnews": DatasetSpec("agnews", "tokens", (128,), 4, 120000, 7600, vocab=30522),
    "sst2": DatasetSpec("sst2", "tokens", (64,), 2, 67349, 872, vocab=30522),
    "imagenet_vit": DatasetSpec("imagenet_vit", "image", (3, 224, 224), 1000, 1281167, 50000),
    "mit-bih": DatasetSpec("mit-bih", "vector", (187,), 5, 87554, 21892),
    "lending_club_loan": DatasetSpec("lending_club_loan", "vector", (90,), 2, 40000, 10000),
    "NUS_WIDE": DatasetSpec("NUS_WIDE", "vector", (1634,), 2, 60000, 40000),
    "UCI_SUSY": DatasetSpec("UCI_SUSY", "vector", (18,), 2, 100000, 20000),
}


def get_spec(name: str) -> DatasetSpec:
    if name in SPECS:
        return SPECS[name]
    low = name.lower()
    for k, v in SPECS.items():
        if k.lower() == low:
            return v
    raise KeyError(f"unknown dataset '{name}'. Known: {sorted(SPECS)}")


class SyntheticGenerator:
    """Deterministic class-conditional sample generator for one dataset spec."""

    def __init__(self, spec: DatasetSpec, seed: int = 0, noise: float = 1.0):
        self.spec = spec
        self.seed = seed
        self.noise = noise
        g = torch.Generator().manual_seed(seed * 7919 + 17)
        k = spec.num_classes
        if spec.kind == "image":
            c, h, w = spec.shape
            # smooth low-frequency class prototypes (upsampled 4x4 noise)
            lo = torch.randn(k, c, 4, 4, generator=g)
            self.proto = torch.nn.functional.interpolate(lo, size=(h, w), mode="bilinear", align_corners=False)
        elif spec.kind in ("vector", "multilabel"):
            d = spec.shape[0]
            self.proto = torch.randn(k, d, generator=g)
        else:  # token kinds
            v = spec.vocab
            logits = torch.randn(k, v, generator=g) * 2.0
            self.token_probs = torch.softmax(logits, dim=1)
            self.trans = None
            if spec.kind == "nwp":
                # a fixed random "next token" map so next-word prediction is learnable
                self.next_tok = torch.randint(0, v, (v,), generator=g)

    def labels(self, n: int, g: torch.Generator, class_probs: Optional[np.ndarray] = None) -> torch.Tensor:
        k = self.spec.num_classes
        if class_probs is None:
            return torch.randint(0, k, (n,), generator=g)
        p = torch.as_tensor(class_probs, dtype=torch.float64)
        return torch.multinomial(p / p.sum(), n, replacement=True, generator=g)

    def sample(self, y: torch.Tensor, g: torch.Generator) -> Tuple[torch.Tensor, torch.Tensor]:
        spec = self.spec
        n = len(y)
        if spec.kind == "image":
            x = 0.5 * self.proto[y] + 0.5 * self.noise * torch.randn((n,) + spec.shape, generator=g)
            return x.float(), y.long()
        if spec.kind == "vector":
            x = self.proto[y] + self.noise * torch.randn((n,) + spec.shape, generator=g)
            if spec.name == "mnist":
                x = torch.sigmoid(x)  # MNIST pixels live in [0, 1]
            return x.float(), y.long()
        if spec.kind == "multilabel":
            x = (torch.rand((n,) + spec.shape, generator=g) < torch.sigmoid(self.proto[y] - 2.0)).float()
            tags = torch.zeros(n, spec.num_classes)
            tags[torch.arange(n), y] = 1.0
            extra = torch.randint(0, spec.num_classes, (n,), generator=g)
            tags[torch.arange(n), extra] = 1.0
            return x, tags
        if spec.kind == "tokens":
            L = spec.shape[0]
            probs = self.token_probs[y]
            toks = torch.multinomial(probs, L, replacement=True, generator=g)
            toks[:, 0] = 101 % spec.vocab  # [CLS]
            return toks.long(), y.long()
        # nwp: x = sequence, y = x shifted by one (next token), 0 = padding
        L = spec.shape[0]
        start = torch.multinomial(self.token_probs[y % self.token_probs.shape[0]], 1, replacement=True,
                                  generator=g).squeeze(1)
        seq = torch.empty(n, L + 1, dtype=torch.long)
        seq[:, 0] = start
        for t in range(1, L + 1):
            rnd = torch.randint(1, spec.vocab, (n,), generator=g)
            keep = torch.rand(n, generator=g) < 0.8
            seq[:, t] = torch.where(keep, self.next_tok[seq[:, t - 1]], rnd)
        seq = seq.clamp_min(1)
        if "shakespeare" in spec.name:
            # character model: predict the single next character (`RNN_OriginalFedAvg` → [B, vocab])
            return seq[:, :L].contiguous(), seq[:, L].contiguous()
        return seq[:, :L].contiguous(), seq[:, 1:].contiguous()

    def make(self, n: int, seed: int, class_probs: Optional[np.ndarray] = None):
        g = torch.Generator().manual_seed(int(seed) & 0x7FFFFFFFFFFF)
        y = self.labels(n, g, class_probs)
        return self.sample(y, g)
