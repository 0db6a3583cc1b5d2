"""TensorFlow-Federated datasets (reference: `data/FederatedEMNIST`, `data/fed_cifar100`,
`data/fed_shakespeare`, `data/stackoverflow_*` — h5 files with ``examples/<client_id>/<field>``).

Two on-disk forms are accepted:
* the TFF ``.h5`` files, when ``h5py`` is importable (it is NOT installed in this image), and
* a pickle-free ``.npz`` conversion with arrays named ``<client_id>/<field>`` (``np.load`` with
  ``allow_pickle=False``), which is what ``convert_h5_to_npz`` writes on a machine that has h5py.

``load_tff_clients(path, x_field, y_field)`` → ``{client_index: (x, y)}`` in sorted client-id order.
"""
import os
from typing import Dict, Tuple

import numpy as np
import torch

_FIELDS = {
    "femnist": ("pixels", "label"), "fed_emnist": ("pixels", "label"), "fed_cifar100": ("image", "label"),
    "fed_shakespeare": ("snippets", None), "stackoverflow_lr": ("tokens", "tags"),
    "stackoverflow_nwp": ("tokens", None),
}


def _from_h5(path, x_field, y_field):
    try:
        import h5py
    except ImportError as e:
        raise ImportError(f"{path}: reading TFF .h5 files needs h5py (not installed here); convert it to .npz "
                          f"with fedml_amd.data.tff.convert_h5_to_npz on a machine that has h5py") from e
    out = {}
    with h5py.File(path, "r") as f:
        ex = f["examples"]
        for i, cid in enumerate(sorted(ex.keys())):
            x = np.asarray(ex[cid][x_field][()])
            y = np.asarray(ex[cid][y_field][()]) if y_field else None
            out[i] = (x, y)
    return out


def _from_npz(path, x_field, y_field):
    data = np.load(path, allow_pickle=False)
    cids = sorted({k.split("/", 1)[0] for k in data.files})
    out = {}
    for i, cid in enumerate(cids):
        x = data[f"{cid}/{x_field}"]
        y = data[f"{cid}/{y_field}"] if y_field and f"{cid}/{y_field}" in data.files else None
        out[i] = (x, y)
    return out


def load_tff_clients(path: str, dataset: str) -> Dict[int, Tuple[torch.Tensor, torch.Tensor]]:
    x_field, y_field = _FIELDS[dataset]
    raw = _from_npz(path, x_field, y_field) if path.endswith(".npz") else _from_h5(path, x_field, y_field)
    out = {}
    for i, (x, y) in raw.items():
        xt = torch.from_numpy(np.ascontiguousarray(x))
        if xt.dtype in (torch.float64,):
            xt = xt.float()
        if dataset == "fed_cifar100" and xt.dim() == 4 and xt.shape[-1] == 3:
            xt = xt.permute(0, 3, 1, 2).float().div(255.0)
        if dataset in ("femnist", "fed_emnist") and xt.dim() == 3:
            xt = xt.unsqueeze(1).float()
        yt = torch.from_numpy(np.ascontiguousarray(y)).long() if y is not None else None
        out[i] = (xt, yt)
    return out


def convert_h5_to_npz(h5_path: str, npz_path: str, dataset: str):  # pragma: no cover - needs h5py
    x_field, y_field = _FIELDS[dataset]
    import h5py
    arrays = {}
    with h5py.File(h5_path, "r") as f:
        for cid in sorted(f["examples"].keys()):
            g = f["examples"][cid]
            arrays[f"{cid}/{x_field}"] = np.asarray(g[x_field][()])
            if y_field:
                arrays[f"{cid}/{y_field}"] = np.asarray(g[y_field][()])
    np.savez(npz_path, **arrays)


def find_tff_file(data_dir: str, dataset: str, train: bool = True):
    names = {"femnist": "fed_emnist", "fed_emnist": "fed_emnist", "fed_cifar100": "fed_cifar100",
             "fed_shakespeare": "shakespeare", "stackoverflow_lr": "stackoverflow", "stackoverflow_nwp": "stackoverflow"}
    base = names.get(dataset, dataset) + ("_train" if train else "_test")
    for ext in (".npz", ".h5"):
        p = os.path.join(data_dir, base + ext)
        if os.path.exists(p):
            return p
    return None
