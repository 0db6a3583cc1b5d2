"""NUS-WIDE vertical-FL parties from the dataset's own files (reference: ``data/NUS_WIDE/nus_wide_dataset.py``).

Layout under ``data_dir`` (the NUS-WIDE distribution):
  Groundtruth/AllLabels/Labels_<concept>.txt            one 0/1 per image (concept frequency → top-k)
  Groundtruth/TrainTestLabels/Labels_<concept>_<Train|Test>.txt
  Low_Level_Features/<Train|Test>_Normalized_<FEATURE>.dat   space-separated image features (party A)
  NUS_WID_Tags/<Train|Test>_Tags1k.dat                  tab-separated 1k tag indicators (party B, or B+C)

Semantics kept from the reference: with several selected concepts only images carrying exactly one of
them are used; the label is +1 for the FIRST selected concept and ``neg_label`` otherwise; both parties
are standardised per column; the first 80 % of the rows train, the rest test; the three-party split
halves the tag columns. Reading is plain numpy (no pandas / sklearn needed)."""
import os
from typing import List, Sequence

import numpy as np


def _read_matrix(path, sep=None):
    rows = []
    with open(path) as f:
        for line in f:
            vals = [v for v in (line.split(sep) if sep else line.split()) if v.strip() != ""]
            if vals:
                rows.append([float(v) for v in vals])
    return np.asarray(rows, dtype=np.float64)


def get_top_k_labels(data_dir: str, top_k: int = 5) -> List[str]:
    d = os.path.join(data_dir, "Groundtruth", "AllLabels")
    counts = {}
    for fn in os.listdir(d):
        p = os.path.join(d, fn)
        if os.path.isfile(p):
            counts[fn[:-4].split("_")[-1]] = int((_read_matrix(p) == 1).sum())
    return [k for k, _ in sorted(counts.items(), key=lambda kv: -kv[1])[:top_k]]


def get_labeled_data(data_dir: str, selected_labels: Sequence[str], n_samples: int = -1, dtype: str = "Train"):
    """(XA image features, XB tags, Y one-hot over the selected concepts) of the usable rows."""
    lab = np.concatenate([_read_matrix(os.path.join(data_dir, "Groundtruth", "TrainTestLabels",
                                                    f"Labels_{c}_{dtype}.txt")) for c in selected_labels], axis=1)
    rows = np.nonzero(lab.sum(1) == 1)[0] if len(selected_labels) > 1 else np.arange(len(lab))
    fdir = os.path.join(data_dir, "Low_Level_Features")
    feats = [_read_matrix(os.path.join(fdir, fn)) for fn in sorted(os.listdir(fdir))
             if fn.startswith(f"{dtype}_Normalized")]
    XA = np.concatenate(feats, axis=1)[rows]
    XB = _read_matrix(os.path.join(data_dir, "NUS_WID_Tags", f"{dtype}_Tags1k.dat"), sep="\t")[rows]
    Y = lab[rows]
    if n_samples != -1:
        XA, XB, Y = XA[:n_samples], XB[:n_samples], Y[:n_samples]
    return XA, XB, Y


def _standardise(X):
    mu, sd = X.mean(0), X.std(0)
    return (X - mu) / np.where(sd > 0, sd, 1.0)


def _binary(Y, neg_label):
    return np.where(Y[:, 0] == 1, 1, neg_label).reshape(-1, 1)


def NUS_WIDE_load_two_party_data(data_dir, selected_labels, neg_label=-1, n_samples=-1):
    XA, XB, Y = get_labeled_data(data_dir, selected_labels, n_samples)
    XA, XB, y = _standardise(XA), _standardise(XB), _binary(Y, neg_label)
    n = int(0.8 * len(XA))
    return [XA[:n], XB[:n], y[:n]], [XA[n:], XB[n:], y[n:]]


def NUS_WIDE_load_three_party_data(data_dir, selected_labels, neg_label=-1, n_samples=-1):
    XA, XB, Y = get_labeled_data(data_dir, selected_labels, n_samples)
    half = XB.shape[1] // 2
    XA, XB, XC, y = _standardise(XA), _standardise(XB[:, :half]), _standardise(XB[:, half:]), _binary(Y, neg_label)
    n = int(0.8 * len(XA))
    return [XA[:n], XB[:n], XC[:n], y[:n]], [XA[n:], XB[n:], XC[n:], y[n:]]
