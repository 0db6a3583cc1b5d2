"""Data loaders: image folders (CINIC/ImageNet layout), Landmarks user CSVs, TFF .npz conversions,
partitioners, and the augmentation reference."""
import csv
import os

import numpy as np
import pytest
import torch

import fedml_amd
from fedml_amd.arguments import Arguments


def _args(**kw):
    cfg = {"training_type": "simulation", "dataset": "mnist", "model": "lr", "client_num_in_total": 2,
           "client_num_per_round": 2, "comm_round": 1, "epochs": 1, "batch_size": 4, "learning_rate": 0.1,
           "backend": "single_process", "federated_optimizer": "FedAvg"}
    cfg.update(kw)
    return fedml_amd.init(Arguments.from_dict({"x": cfg}))


def _png(path, color, size=(40, 48)):
    from PIL import Image
    os.makedirs(os.path.dirname(path), exist_ok=True)
    Image.new("RGB", size, color).save(path)


def test_image_folder_cinic_layout(tmp_path):
    for split in ("train", "test"):
        for ci, (cname, color) in enumerate((("cat", (255, 0, 0)), ("dog", (0, 0, 255)))):
            for i in range(4):
                _png(str(tmp_path / split / cname / f"{i}.png"), color)
    a = _args(dataset="cinic10", data_cache_dir=str(tmp_path), partition_method="homo")
    ds, k = fedml_amd.data.load(a)
    assert k == 2 and ds[0] == 8
    x, y = next(iter(ds[5][0]))
    assert x.shape[1:] == (3, 32, 32)
    # red images → high normalised R channel, blue → high B channel
    xs, ys = ds[2].x, ds[2].y
    assert float(xs[ys == 0][:, 0].mean()) > float(xs[ys == 0][:, 2].mean())


def test_landmarks_user_partition(tmp_path):
    os.makedirs(tmp_path / "data_user_dict")
    rows = [("0", "a", 0), ("0", "b", 1), ("1", "c", 1), ("2", "d", 0), ("2", "e", 2)]
    for split in ("train", "test"):
        with open(tmp_path / "data_user_dict" / f"gld23k_user_dict_{split}.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["user_id", "image_id", "class"])
            w.writerows(rows)
    for _, img, cls in rows:
        _png(str(tmp_path / "images" / f"{img}.jpg"), (cls * 80, 10, 10))
    a = _args(dataset="gld23k", data_cache_dir=str(tmp_path), image_size=16, client_num_in_total=9)
    ds, k = fedml_amd.data.load(a)
    assert a.client_num_in_total == 3
    assert [ds[4][c] for c in range(3)] == [2, 1, 2]


def test_tff_npz(tmp_path):
    rng = np.random.RandomState(0)
    arrays = {}
    for cid, n in (("f0001", 5), ("f0002", 3)):
        arrays[f"{cid}/pixels"] = rng.rand(n, 28, 28).astype(np.float32)
        arrays[f"{cid}/label"] = rng.randint(0, 62, size=n).astype(np.int32)
    np.savez(tmp_path / "fed_emnist_train.npz", **arrays)
    np.savez(tmp_path / "fed_emnist_test.npz", **arrays)
    a = _args(dataset="femnist", model="cnn", data_cache_dir=str(tmp_path), client_num_in_total=100)
    ds, k = fedml_amd.data.load(a)
    assert a.client_num_in_total == 2 and ds[4] == {0: 5, 1: 3}
    x, y = next(iter(ds[5][0]))
    assert x.shape[1:] == (1, 28, 28)


def test_tff_h5_without_h5py_is_explicit(tmp_path):
    from fedml_amd.data.tff import load_tff_clients
    p = tmp_path / "x.h5"
    p.write_bytes(b"not really h5")
    try:
        import h5py  # noqa: F401
        pytest.skip("h5py present")
    except ImportError:
        with pytest.raises(ImportError, match="h5py"):
            load_tff_clients(str(p), "femnist")


def test_dirichlet_partition_reference_properties():
    from fedml_amd.core.non_iid_partition import non_iid_partition_with_dirichlet_distribution
    np.random.seed(10)
    labels = np.random.randint(0, 10, size=5000)
    parts = non_iid_partition_with_dirichlet_distribution(labels, 20, 10, 0.5)
    allidx = np.concatenate([np.asarray(v) for v in parts.values()])
    assert len(allidx) == 5000 and len(np.unique(allidx)) == 5000
    assert min(len(v) for v in parts.values()) >= 10


def test_augment_cpu_reference_semantics():
    from fedml_amd import ops
    x = torch.arange(2 * 1 * 8 * 8, dtype=torch.float32).view(2, 1, 8, 8)
    y = ops.augment(x, seed=1, pad=0, cutout=0, flip=False)
    assert torch.equal(x, y)
    z = ops.augment(x, seed=1, pad=2, cutout=4, flip=True)
    assert z.shape == x.shape and (z == 0).any()
