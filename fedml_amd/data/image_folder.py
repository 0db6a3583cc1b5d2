"""Image-folder datasets (reference: `data/ImageNet/*`, `data/Landmarks/*`, `data/cinic10/*`).

* ``load_image_folder(root)`` — ``root/<class_name>/<image>`` trees (ImageNet ILSVRC2012 train/val,
  CINIC-10 train/test): decoded with PIL, resized (shorter side) + centre-cropped to ``size``,
  normalised; returns uint8-free fp32 tensors [N, 3, size, size] and int64 labels.
* ``load_landmarks(root, split)`` — Google Landmarks gld23k / gld160k: the federated split comes
  from the user-dict CSVs (``user_id,image_id,class``); images are ``images/<image_id>.jpg``.
  Returns ``{client_id: (x, y)}`` with clients = users (the reference's natural partition).

Decoding happens once, on the host, into tensors; training then reads the HBM-resident client
store, and augmentation runs on the device (``ops.augment``).
"""
import csv
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

_IMAGENET_MEAN = (0.485, 0.456, 0.406)
_IMAGENET_STD = (0.229, 0.224, 0.225)
_EXT = (".jpg", ".jpeg", ".png", ".bmp", ".webp")


def _decode(path, size):
    from PIL import Image
    with Image.open(path) as im:
        im = im.convert("RGB")
        w, h = im.size
        s = size / min(w, h)
        im = im.resize((max(size, round(w * s)), max(size, round(h * s))), Image.BILINEAR)
        w, h = im.size
        l, t = (w - size) // 2, (h - size) // 2
        im = im.crop((l, t, l + size, t + size))
        return np.asarray(im, dtype=np.uint8)


def _to_tensor(arrs: List[np.ndarray], mean, std):
    x = torch.from_numpy(np.stack(arrs)).permute(0, 3, 1, 2).float().div_(255.0)
    m = torch.tensor(mean).view(1, 3, 1, 1)
    sd = torch.tensor(std).view(1, 3, 1, 1)
    return (x - m) / sd


def load_image_folder(root: str, size: int = 224, max_per_class: Optional[int] = None, mean=_IMAGENET_MEAN,
                      std=_IMAGENET_STD) -> Tuple[torch.Tensor, torch.Tensor, List[str]]:
    classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
    arrs, labels = [], []
    for ci, cname in enumerate(classes):
        files = sorted(f for f in os.listdir(os.path.join(root, cname)) if f.lower().endswith(_EXT))
        if max_per_class:
            files = files[:max_per_class]
        for f in files:
            arrs.append(_decode(os.path.join(root, cname, f), size))
            labels.append(ci)
    if not arrs:
        raise FileNotFoundError(f"no images under {root}")
    return _to_tensor(arrs, mean, std), torch.tensor(labels, dtype=torch.int64), classes


def load_landmarks(root: str, split: str = "gld23k", size: int = 224, train: bool = True
                   ) -> Dict[int, Tuple[torch.Tensor, torch.Tensor]]:
    name = f"{split}_user_dict_{'train' if train else 'test'}.csv"
    cands = [os.path.join(root, "data_user_dict", name), os.path.join(root, name)]
    csv_path = next((c for c in cands if os.path.exists(c)), None)
    if csv_path is None:
        raise FileNotFoundError(f"{name} not found under {root}")
    per_user: Dict[str, List[Tuple[str, int]]] = {}
    with open(csv_path) as f:
        for row in csv.DictReader(f):
            per_user.setdefault(row["user_id"], []).append((row["image_id"], int(row["class"])))
    img_dir = os.path.join(root, "images")
    out = {}
    for cid, user in enumerate(sorted(per_user, key=lambda u: int(u) if u.isdigit() else u)):
        arrs, ys = [], []
        for image_id, cls in per_user[user]:
            p = os.path.join(img_dir, image_id + ".jpg")
            if not os.path.exists(p):
                continue
            arrs.append(_decode(p, size))
            ys.append(cls)
        if arrs:
            out[cid] = (_to_tensor(arrs, _IMAGENET_MEAN, _IMAGENET_STD), torch.tensor(ys, dtype=torch.int64))
    return out
