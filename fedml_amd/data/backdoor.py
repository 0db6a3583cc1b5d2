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


# ---------------------------------------------------------------------------------------------------
# Edge-case (out-of-distribution) backdoors with REAL edge-case images (reference
# data/edge_case_examples/data_loader.py:319-640 — Southwest airliners labelled "truck" (9) on CIFAR-10,
# ARDIS sevens labelled "1" on EMNIST/MNIST). The reference ships those images as pickles and full-object
# ``torch.load`` files; here they are read only through loaders that execute nothing from the file:
# ``.npy`` (allow_pickle=False), ``.npz`` arrays or safetensors (key ``images``), uint8 [N, H, W(, C)].
# ---------------------------------------------------------------------------------------------------
EDGE_CASE_TARGETS = {"southwest": 9, "ardis": 1}


def load_edge_case_images(path: str):
    import numpy as np
    if path.endswith(".npy"):
        a = np.load(path, allow_pickle=False)
    elif path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            a = z["images"] if "images" in z else z[list(z.keys())[0]]
    elif path.endswith(".safetensors"):
        from safetensors.numpy import load_file
        a = load_file(path)["images"]
    else:
        raise ValueError(f"{path}: edge-case images must be .npy / .npz / .safetensors (pickles are refused)")
    return torch.from_numpy(np.ascontiguousarray(a))


def _to_nchw_float(img: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
    x = img.float()
    if x.dim() == 3:                       # [N, H, W] grey
        x = x.unsqueeze(1)
    elif x.dim() == 4 and x.shape[-1] in (1, 3) and x.shape[1] not in (1, 3):
        x = x.permute(0, 3, 1, 2)          # NHWC → NCHW
    if x.max() > 1.5:
        x = x / 255.0
    return x.reshape(x.shape[0], *like.shape[1:]) if x[0].numel() == like[0].numel() else x


def edge_case_poisoned_set(clean: ClientData, edge_train: torch.Tensor, poison_type: str = "southwest",
                           attack_case: str = "edge-case", n_edge: int = 100, n_clean: int = 400, seed: int = 0):
    """The attacker's training set: ``n_clean`` random clean samples + ``n_edge`` edge-case images
    relabelled to the poison target (``normal-case``/``almost-edge-case`` keep all edge-case images
    and sample clean ones only, as the reference)."""
    g = torch.Generator().manual_seed(seed)
    target = EDGE_CASE_TARGETS[poison_type]
    ex = _to_nchw_float(edge_train, clean.x)
    if attack_case == "edge-case" and len(ex) > n_edge:
        ex = ex[torch.randperm(len(ex), generator=g)[:n_edge]]
    ci = torch.randperm(clean.num_samples, generator=g)[:min(n_clean, clean.num_samples)]
    x = torch.cat([clean.x[ci].float(), ex.to(clean.x.device)])
    y = torch.cat([clean.y[ci], torch.full((len(ex),), target, dtype=clean.y.dtype, device=clean.y.device)])
    return ClientData(x, y, clean.batch_size, shuffle=True, seed=seed)


def edge_case_test_set(edge_test: torch.Tensor, like: ClientData, poison_type: str = "southwest"):
    """Targeted-task test set: every edge-case test image labelled with the poison target."""
    ex = _to_nchw_float(edge_test, like.x)
    return ClientData(ex, torch.full((len(ex),), EDGE_CASE_TARGETS[poison_type], dtype=like.y.dtype), like.batch_size)
