"""Small metric helpers (no sklearn dependency on the hot path)."""
import torch


def roc_auc(scores: torch.Tensor, labels: torch.Tensor) -> float:
    """Rank-based ROC AUC (Mann–Whitney U); ties receive their average rank."""
    s = scores.detach().double().reshape(-1).cpu()
    labels = labels.detach().reshape(-1).cpu()
    order = torch.argsort(s)
    ranks = torch.empty_like(s)
    ranks[order] = torch.arange(1, len(s) + 1, dtype=s.dtype)
    uniq, inv = torch.unique(s, return_inverse=True)
    if len(uniq) < len(s):
        sums = torch.zeros(len(uniq), dtype=s.dtype).index_add_(0, inv, ranks)
        cnt = torch.zeros(len(uniq), dtype=s.dtype).index_add_(0, inv, torch.ones_like(s))
        ranks = (sums / cnt)[inv]
    pos = labels > 0.5
    n1, n0 = int(pos.sum()), int((~pos).sum())
    if n1 == 0 or n0 == 0:
        return float("nan")
    return float((ranks[pos].sum() - n1 * (n1 + 1) / 2) / (n1 * n0))


def binary_prf(pred: torch.Tensor, target: torch.Tensor):
    """Macro precision / recall / F1 over the two classes of a binary prediction."""
    out = []
    for c in (0, 1):
        tp = float(((pred == c) & (target == c)).sum())
        fp = float(((pred == c) & (target != c)).sum())
        fn = float(((pred != c) & (target == c)).sum())
        p = tp / (tp + fp) if tp + fp else 0.0
        r = tp / (tp + fn) if tp + fn else 0.0
        out.append((p, r, 2 * p * r / (p + r) if p + r else 0.0))
    return tuple(sum(v[i] for v in out) / 2 for i in range(3))
