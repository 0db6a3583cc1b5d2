"""``fedml_amd.data.load(args)`` → the reference's 8-tuple contract.

Return value (parity with `data/data_loader.py:312-322`):
    ([train_data_num, test_data_num, train_data_global, test_data_global,
      train_data_local_num_dict, train_data_local_dict, test_data_local_dict, class_num], class_num)

Sources, in order:
  1. real LEAF-JSON MNIST under ``data_cache_dir/{train,test}`` (natural user partition,
     `np.random.seed(100)` batch shuffling as `data/MNIST/data_loader.py:75-98`);
  2. real CIFAR-10/100 binary batches under ``data_cache_dir`` (no pickle);
  3. otherwise (or with ``synthetic_data: true``) the synthetic twin of the dataset
     (``data/synthetic.py``) partitioned homo / hetero (LDA, `np.random.seed(10)` as
     `data/cifar10/data_loader.py:123`).
Centralized mode (``client_num_in_total == 1`` outside cross-silo) and full-batch mode
(``batch_size <= 0``) follow `data/data_loader.py:276-310`.
"""
import json
import logging
import os
from typing import Dict, List

import numpy as np
import torch

from ..core.non_iid_partition import homo_partition, non_iid_partition_with_dirichlet_distribution
from .client_data import ClientData, concat_client_data, split_client_data
from .synthetic import SyntheticGenerator, get_spec


def _leaf_dirs(args):
    base = getattr(args, "data_cache_dir", "") or ""
    for tr, te in ((os.path.join(base, "train"), os.path.join(base, "test")),
                   (os.path.join(base, "MNIST", "train"), os.path.join(base, "MNIST", "test"))):
        if os.path.isdir(tr) and os.path.isdir(te) and any(f.endswith(".json") for f in os.listdir(tr)):
            return tr, te
    return None


def read_leaf(train_dir, test_dir):
    users, train, test = [], {}, {}
    for f in sorted(os.listdir(train_dir)):
        if f.endswith(".json"):
            with open(os.path.join(train_dir, f)) as fh:
                d = json.load(fh)
            users.extend(d["users"])
            train.update(d["user_data"])
    for f in sorted(os.listdir(test_dir)):
        if f.endswith(".json"):
            with open(os.path.join(test_dir, f)) as fh:
                test.update(json.load(fh)["user_data"])
    return sorted(users), train, test


def _leaf_batches(data, batch_size):
    """Reference batching: seed 100, shuffle x and y with the same RNG state. Text clients (LEAF
    Shakespeare: 80-character strings → next character) go through the character vocabulary
    (``shakespeare.process_x/process_y``, reference ``data/shakespeare/data_loader.py:53-63``)."""
    from .shakespeare import is_char_data, process_x, process_y
    if is_char_data(data["x"]):
        x = process_x(data["x"])
        y = process_y(data["y"])
    else:
        x = np.asarray(data["x"], dtype=np.float32)
        y = np.asarray(data["y"], dtype=np.int64)
    np.random.seed(100)
    state = np.random.get_state()
    np.random.shuffle(x)
    np.random.set_state(state)
    np.random.shuffle(y)
    return ClientData(torch.from_numpy(x), torch.from_numpy(y), batch_size)


def _load_leaf(args, train_dir, test_dir, class_num):
    users, train, test = read_leaf(train_dir, test_dir)
    tl, te, nd = {}, {}, {}
    for cid, u in enumerate(users):
        tl[cid] = _leaf_batches(train[u], args.batch_size)
        te[cid] = _leaf_batches(test[u], args.batch_size)
        nd[cid] = tl[cid].num_samples
    return tl, te, nd, class_num


def _read_cifar_bin(base, name):
    """CIFAR binary format (`cifar-10-batches-bin`, `cifar-100-binary`): uint8 records, no pickle."""
    if name == "cifar10":
        d = os.path.join(base, "cifar-10-batches-bin")
        tr_files = [os.path.join(d, f"data_batch_{i}.bin") for i in range(1, 6)]
        te_files = [os.path.join(d, "test_batch.bin")]
        lbl_bytes, lbl_off = 1, 0
    else:
        d = os.path.join(base, "cifar-100-binary")
        tr_files, te_files = [os.path.join(d, "train.bin")], [os.path.join(d, "test.bin")]
        lbl_bytes, lbl_off = 2, 1
    if not all(os.path.exists(f) for f in tr_files + te_files):
        return None

    def rd(files):
        raw = np.concatenate([np.fromfile(f, dtype=np.uint8) for f in files])
        rec = raw.reshape(-1, lbl_bytes + 3072)
        y = rec[:, lbl_off].astype(np.int64)
        x = rec[:, lbl_bytes:].reshape(-1, 3, 32, 32).astype(np.float32) / 255.0
        mean = np.array([0.4914, 0.4822, 0.4465], dtype=np.float32).reshape(1, 3, 1, 1)
        std = np.array([0.2470, 0.2435, 0.2616], dtype=np.float32).reshape(1, 3, 1, 1)
        return torch.from_numpy((x - mean) / std), torch.from_numpy(y)

    return rd(tr_files), rd(te_files)


def _partition(labels: np.ndarray, client_num: int, method: str, alpha: float, class_num: int) -> Dict[int, List[int]]:
    np.random.seed(10)
    if method in ("homo", "iid"):
        return {k: list(v) for k, v in homo_partition(len(labels), client_num).items()}
    return non_iid_partition_with_dirichlet_distribution(labels, client_num, class_num, alpha)


def _load_synthetic(args, spec):
    client_num = int(args.client_num_in_total)
    per_client = int(getattr(args, "synthetic_train_samples_per_client", 0) or 0)
    if per_client <= 0:
        per_client = max(20, min(600, spec.train_size // max(client_num, 1)))
    n_train = per_client * client_num
    test_per_client = int(getattr(args, "synthetic_test_samples_per_client", 0) or max(10, per_client // 5))
    seed = int(getattr(args, "random_seed", 0))
    gen = SyntheticGenerator(spec, seed=seed, noise=float(getattr(args, "synthetic_noise", 1.0)))
    # balanced global label list, then the reference partitioner
    rng = np.random.RandomState(seed + 1234)
    labels = rng.randint(0, spec.num_classes, size=n_train)
    method = getattr(args, "partition_method", "hetero")
    alpha = float(getattr(args, "partition_alpha", 0.5))
    if client_num == 1:
        parts = {0: list(range(n_train))}
    else:
        parts = _partition(labels, client_num, method, alpha, spec.num_classes)
    tl, te, nd = {}, {}, {}
    for cid in range(client_num):
        idx = np.asarray(parts[cid], dtype=np.int64)
        y = torch.as_tensor(labels[idx]) if spec.kind not in ("nwp",) else torch.zeros(len(idx), dtype=torch.long)
        g = torch.Generator().manual_seed(seed * 1000003 + cid * 7 + 1)
        if spec.kind == "nwp":
            x, yy = gen.sample(y, g)
        else:
            x, yy = gen.sample(y, g)
        tl[cid] = ClientData(x, yy, args.batch_size)
        nd[cid] = len(idx)
        # IID test set per client
        gt = torch.Generator().manual_seed(seed * 1000003 + cid * 7 + 5)
        yt = gen.labels(test_per_client, gt)
        xt, ytt = gen.sample(yt, gt)
        te[cid] = ClientData(xt, ytt, args.batch_size)
    return tl, te, nd, spec.num_classes


def _clients_to_loaded(train: Dict[int, tuple], test: Dict[int, tuple], bs, class_num):
    tl = {c: ClientData(x, y, bs, shuffle=True, seed=c) for c, (x, y) in train.items()}
    te = {c: ClientData(x, y, bs) for c, (x, y) in test.items()} if test else {
        c: ClientData(tl[c].x[:0], tl[c].y[:0], bs) for c in tl}
    return tl, te, {c: d.num_samples for c, d in tl.items()}, class_num


def _load_files(args, name, spec):
    """Real files when present: TFF (.npz / .h5), image folders (ImageNet, CINIC-10), Landmarks CSVs."""
    base = getattr(args, "data_cache_dir", "") or ""
    bs = args.batch_size
    try:
        if name in ("femnist", "fed_emnist", "fed_cifar100", "fed_shakespeare", "stackoverflow_lr",
                    "stackoverflow_nwp"):
            from .tff import find_tff_file, load_tff_clients
            tr, te = find_tff_file(base, name, True), find_tff_file(base, name, False)
            if tr:
                train = load_tff_clients(tr, name)
                test = load_tff_clients(te, name) if te else {}
                args.client_num_in_total = len(train)
                return _clients_to_loaded(train, test, bs, spec.num_classes)
        if name in ("ILSVRC2012", "ILSVRC2012_hdf5", "cinic10") and os.path.isdir(os.path.join(base, "train")):
            from .image_folder import load_image_folder
            size = 32 if name == "cinic10" else int(getattr(args, "image_size", 224))
            xtr, ytr, classes = load_image_folder(os.path.join(base, "train"), size,
                                                  getattr(args, "max_images_per_class", None))
            val_dir = next((os.path.join(base, d) for d in ("val", "test", "valid") if
                            os.path.isdir(os.path.join(base, d))), None)
            parts = _partition(ytr.numpy(), int(args.client_num_in_total), args.partition_method,
                               float(args.partition_alpha), len(classes))
            train = {c: (xtr[torch.as_tensor(v, dtype=torch.long)], ytr[torch.as_tensor(v, dtype=torch.long)])
                     for c, v in parts.items()}
            test = {}
            if val_dir:
                xte, yte, _ = load_image_folder(val_dir, size, getattr(args, "max_images_per_class", None))
                for c, v in enumerate(np.array_split(np.arange(len(yte)), int(args.client_num_in_total))):
                    test[c] = (xte[torch.as_tensor(v, dtype=torch.long)], yte[torch.as_tensor(v, dtype=torch.long)])
            return _clients_to_loaded(train, test, bs, len(classes))
        if name in ("gld23k", "gld160k"):
            from .image_folder import load_landmarks
            train = load_landmarks(base, name, int(getattr(args, "image_size", 224)), True)
            test = load_landmarks(base, name, int(getattr(args, "image_size", 224)), False)
            if train:
                args.client_num_in_total = len(train)
                return _clients_to_loaded(train, test, bs, spec.num_classes)
    except FileNotFoundError:
        return None
    return None


def load_synthetic_data(args):
    dataset_name = args.dataset
    centralized = int(args.client_num_in_total) == 1 and getattr(args, "training_type", "") != "cross_silo"
    args_batch_size = args.batch_size
    full_batch = args.batch_size is None or int(args.batch_size) <= 0
    if full_batch:
        args.batch_size = 128
    spec = get_spec(dataset_name)
    force_syn = bool(getattr(args, "synthetic_data", False))
    loaded = None
    if not force_syn and dataset_name in ("mnist", "femnist", "shakespeare"):
        dirs = _leaf_dirs(args)
        if dirs is not None:
            loaded = _load_leaf(args, dirs[0], dirs[1], spec.num_classes)
            args.client_num_in_total = len(loaded[0])
    if loaded is None and not force_syn and dataset_name in ("cifar10", "cifar100"):
        real = _read_cifar_bin(getattr(args, "data_cache_dir", ""), dataset_name)
        if real is not None:
            (xtr, ytr), (xte, yte) = real
            parts = _partition(ytr.numpy(), int(args.client_num_in_total), args.partition_method,
                               float(args.partition_alpha), spec.num_classes)
            tl = {c: ClientData(xtr[torch.as_tensor(v)], ytr[torch.as_tensor(v)], args.batch_size, shuffle=True,
                                seed=c) for c, v in parts.items()}
            nd = {c: len(v) for c, v in parts.items()}
            te_parts = np.array_split(np.arange(len(yte)), int(args.client_num_in_total))
            te = {c: ClientData(xte[torch.as_tensor(v)], yte[torch.as_tensor(v)], args.batch_size)
                  for c, v in enumerate(te_parts)}
            loaded = (tl, te, nd, spec.num_classes)
    if loaded is None and not force_syn:
        loaded = _load_files(args, dataset_name, spec)
    if loaded is None:
        if not force_syn:
            logging.info("dataset %s: no local files under %s → synthetic data of the same shape", dataset_name,
                         getattr(args, "data_cache_dir", ""))
        loaded = _load_synthetic(args, spec)
    train_local, test_local, num_dict, class_num = loaded

    if centralized and len(train_local) > 1:
        train_local = {0: concat_client_data([train_local[c] for c in sorted(train_local)])}
        test_local = {0: concat_client_data([test_local[c] for c in sorted(test_local)])}
        num_dict = {0: train_local[0].num_samples}
        args.client_num_in_total = 1

    if full_batch:
        train_local = {c: d.with_batch_size(max(1, d.num_samples)) for c, d in train_local.items()}
        test_local = {c: d.with_batch_size(max(1, d.num_samples)) for c, d in test_local.items()}
        args.batch_size = args_batch_size

    train_global = concat_client_data([train_local[c] for c in sorted(train_local)],
                                      batch_size=None if not full_batch else None)
    test_global = concat_client_data([test_local[c] for c in sorted(test_local)])
    if full_batch:
        train_global = train_global.with_batch_size(max(1, train_global.num_samples))
        test_global = test_global.with_batch_size(max(1, test_global.num_samples))
    train_num = sum(num_dict.values())
    test_num = test_global.num_samples
    dataset = [train_num, test_num, train_global, test_global, num_dict, train_local, test_local, class_num]
    return dataset, class_num


def load(args):
    return load_synthetic_data(args)


def load_cross_silo(args):
    """Like ``load`` but each client's train data is sharded over the silo's data-parallel
    processes (``n_proc_in_silo``): ``train_data_local_dict[cid]`` becomes a list of shards
    (reference: `data/data_loader_cross_silo.py:58-86`)."""
    dataset, class_num = load_synthetic_data(args)
    n = int(getattr(args, "n_proc_in_silo", 1) or 1)
    dataset[5] = {cid: split_client_data(cd, n) for cid, cd in dataset[5].items()}
    return dataset, class_num


def merge_to_centralized(dataset):
    """Collapse a federated 8-tuple into its 1-client centralized twin (for the FedAvg ≡ centralized check)."""
    train_num, test_num, tg, teg, nd, tl, tel, k = dataset
    bs = tl[sorted(tl)[0]].batch_size
    merged = concat_client_data([tl[c] for c in sorted(tl)], batch_size=bs)
    merged_te = concat_client_data([tel[c] for c in sorted(tel)], batch_size=bs)
    return [train_num, test_num, tg, teg, {0: merged.num_samples}, {0: merged}, {0: merged_te}, k]
