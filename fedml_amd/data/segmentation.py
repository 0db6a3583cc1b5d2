"""Synthetic federated segmentation data (stand-in for Pascal VOC / COCO / Cityscapes shards used
by the reference's FedSeg — no dataset downloads are possible here). Each image holds a few
axis-aligned objects whose class determines a colour signature; the mask labels each pixel with
its class and marks a 1-pixel border as ``255`` (ignore), like VOC's boundary annotations."""
import numpy as np
import torch

from .client_data import ClientData


def _make(n, hw, n_classes, rng):
    x = rng.normal(0, 0.3, size=(n, 3, hw, hw)).astype(np.float32)
    y = np.zeros((n, hw, hw), dtype=np.int64)
    palette = rng.uniform(-1.5, 1.5, size=(n_classes, 3)).astype(np.float32)
    for i in range(n):
        for _ in range(rng.integers(1, 4)):
            c = int(rng.integers(1, n_classes))
            h, w = rng.integers(hw // 6, hw // 2, size=2)
            r0, c0 = rng.integers(0, hw - h), rng.integers(0, hw - w)
            x[i, :, r0:r0 + h, c0:c0 + w] += palette[c][:, None, None]
            y[i, r0:r0 + h, c0:c0 + w] = c
            y[i, r0, c0:c0 + w] = 255
            y[i, r0 + h - 1, c0:c0 + w] = 255
    return torch.from_numpy(x), torch.from_numpy(y)


def load_synthetic_segmentation(client_num, samples_per_client=16, n_classes=6, hw=32, batch_size=4, seed=0):
    rng = np.random.default_rng(seed)
    train_local, test_local, nums = {}, {}, {}
    trs, tes = [], []
    for c in range(client_num):
        xtr, ytr = _make(samples_per_client, hw, n_classes, rng)
        xte, yte = _make(max(2, samples_per_client // 4), hw, n_classes, rng)
        train_local[c] = ClientData(xtr, ytr, batch_size, shuffle=True, seed=seed + c)
        test_local[c] = ClientData(xte, yte, batch_size)
        nums[c] = samples_per_client
        trs.append((xtr, ytr))
        tes.append((xte, yte))
    gtr = ClientData(torch.cat([a for a, _ in trs]), torch.cat([b for _, b in trs]), batch_size)
    gte = ClientData(torch.cat([a for a, _ in tes]), torch.cat([b for _, b in tes]), batch_size)
    return [gtr.num_samples, gte.num_samples, gtr, gte, nums, train_local, test_local, n_classes], n_classes
