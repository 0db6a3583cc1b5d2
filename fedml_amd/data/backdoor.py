"""Backdoor / edge-case poisoning data (reference B7: `data/edge_case_examples/*` — ARDIS, southwest,
"greencar" poisoned sets for the robust-FedAvg attack experiments).

The reference downloads real edge-case images; here a trigger-pattern backdoor is synthesised
on any image/vector client dataset: a fixed corner patch (images) or a fixed feature pattern
(vectors) is stamped onto a fraction of samples whose labels are flipped to ``target_label``."""
import torch

from .client_data import ClientData


def stamp_trigger(x: torch.Tensor, value: float = 3.0) -> torch.Tensor:
    x = x.clone()
    if x.dim() == 4:        # [N, C, H, W]: 3×3 bottom-right patch
        x[:, :, -3:, -3:] = value
    elif x.dim() == 3:      # [N, H, W]
        x[:, -3:, -3:] = value
    else:                   # [N, D]: last 16 features
        x[:, -16:] = value
    return x


def poison_client_data(cd: ClientData, target_label: int = 0, fraction: float = 0.5, seed: int = 0) -> ClientData:
    g = torch.Generator().manual_seed(seed)
    n = cd.num_samples
    k = int(n * fraction)
    idx = torch.randperm(n, generator=g)[:k]
    x = cd.x.clone()
    y = cd.y.clone()
    x[idx] = stamp_trigger(cd.x[idx])
    y[idx] = target_label
    return ClientData(x, y, cd.batch_size, cd.shuffle, cd.seed)


def backdoor_test_set(cd: ClientData, target_label: int = 0) -> ClientData:
    """All test samples (excluding the target class) triggered and labelled with the target."""
    keep = cd.y != target_label
    x = stamp_trigger(cd.x[keep])
    y = torch.full((int(keep.sum()),), target_label, dtype=cd.y.dtype)
    return ClientData(x, y, cd.batch_size)
