"""Latent-Dirichlet (LDA) label partition and homogeneous split.

Reproduces the RNG call sequence of `core/non_iid_partition/noniid_partition.py:6-109`
(per class: shuffle idx_k, draw a Dirichlet proportion, zero out clients that
already hold ≥ N/client_num samples, split; repeat until every client has ≥ 10
samples; finally shuffle each client's list), so that for the same global
``np.random`` state the client → indices map is identical to the reference.
"""
import logging

import numpy as np


def partition_class_samples_with_dirichlet_distribution(N, alpha, client_num, idx_batch, idx_k):
    np.random.shuffle(idx_k)
    proportions = np.random.dirichlet(np.repeat(alpha, client_num))
    sizes = np.fromiter((len(b) for b in idx_batch), dtype=np.int64, count=client_num)
    proportions = proportions * (sizes < N / client_num)
    proportions = proportions / proportions.sum()
    cuts = (np.cumsum(proportions) * len(idx_k)).astype(int)[:-1]
    idx_batch = [b + part.tolist() for b, part in zip(idx_batch, np.split(idx_k, cuts))]
    return idx_batch, min(len(b) for b in idx_batch)


def non_iid_partition_with_dirichlet_distribution(label_list, client_num, classes, alpha, task="classification",
                                                  min_require_size=10):
    label_list = label_list if task == "segmentation" else np.asarray(label_list)
    N = len(label_list)
    min_size = 0
    while min_size < min_require_size:
        idx_batch = [[] for _ in range(client_num)]
        if task == "segmentation":
            for c, cat in enumerate(classes):
                if c > 0:
                    mask = [np.any(label_list[i] == cat) and not np.any(np.in1d(label_list[i], classes[:c]))
                            for i in range(N)]
                else:
                    mask = [np.any(label_list[i] == cat) for i in range(N)]
                idx_k = np.where(np.asarray(mask))[0]
                idx_batch, min_size = partition_class_samples_with_dirichlet_distribution(
                    N, alpha, client_num, idx_batch, idx_k)
        else:
            for k in range(classes):
                idx_k = np.where(label_list == k)[0]
                idx_batch, min_size = partition_class_samples_with_dirichlet_distribution(
                    N, alpha, client_num, idx_batch, idx_k)
    net_dataidx_map = {}
    for i in range(client_num):
        np.random.shuffle(idx_batch[i])
        net_dataidx_map[i] = idx_batch[i]
    return net_dataidx_map


def homo_partition(n_samples, client_num):
    """IID split: random permutation cut into ``client_num`` near-equal parts
    (reference: `data/cifar10/data_loader.py:129-133`)."""
    idxs = np.random.permutation(n_samples)
    batch_idxs = np.array_split(idxs, client_num)
    return {i: batch_idxs[i] for i in range(client_num)}


def record_data_stats(y_train, net_dataidx_map, task="classification"):
    net_cls_counts = {}
    for net_i, dataidx in net_dataidx_map.items():
        if task == "segmentation":
            unq, cnt = np.unique(np.concatenate(y_train[dataidx]), return_counts=True)
        else:
            unq, cnt = np.unique(np.asarray(y_train)[dataidx], return_counts=True)
        net_cls_counts[net_i] = {int(u): int(c) for u, c in zip(unq, cnt)}
    logging.debug("Data statistics: %s", net_cls_counts)
    return net_cls_counts
