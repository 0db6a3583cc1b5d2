"""NUS-WIDE party loader on a miniature copy of the dataset's file layout (the real files are not
available offline; parity of the file semantics with data/NUS_WIDE/nus_wide_dataset.py)."""
import numpy as np

from fedml_amd.data.nus_wide import NUS_WIDE_load_three_party_data, NUS_WIDE_load_two_party_data, get_top_k_labels


def _make(root, n=20, rng=np.random.default_rng(0)):
    gt, tt = root / "Groundtruth" / "AllLabels", root / "Groundtruth" / "TrainTestLabels"
    lf, tg = root / "Low_Level_Features", root / "NUS_WID_Tags"
    for d in (gt, tt, lf, tg):
        d.mkdir(parents=True)
    which = rng.integers(0, 3, n)                   # concept per image: sky / water / person
    for j, c in enumerate(("sky", "water", "person")):
        lab = (which == j).astype(int)
        if j == 1:
            lab[0] = 1                              # image 0 carries two concepts → dropped
        (gt / f"Labels_{c}.txt").write_text("\n".join(map(str, np.r_[lab, [j == 0] * (5 - j)].astype(int))) + "\n")
        (tt / f"Labels_{c}_Train.txt").write_text("\n".join(map(str, lab)) + "\n")
    for name, d in (("CH", 4), ("EDH", 3)):
        (lf / f"Train_Normalized_{name}.dat").write_text(
            "\n".join(" ".join(f"{v:.4f}" for v in rng.normal(size=d)) + " " for _ in range(n)) + "\n")
    (tg / "Train_Tags1k.dat").write_text("\n".join("\t".join(str(int(v)) for v in rng.integers(0, 2, 6)) + "\t"
                                                   for _ in range(n)) + "\n")
    return which


def test_two_and_three_party_parsing(tmp_path):
    which = _make(tmp_path)
    assert get_top_k_labels(str(tmp_path), 1) == ["sky"]
    (xa, xb, y), (xa_t, xb_t, y_t) = NUS_WIDE_load_two_party_data(str(tmp_path), ["sky", "water", "person"])
    rows = [i for i in range(len(which)) if i != 0 or which[0] == 1]   # row 0 dropped unless it was water only
    n = len(rows)
    assert len(xa) + len(xa_t) == n and xa.shape[1] == 7 and xb.shape[1] == 6
    assert set(np.unique(np.r_[y[:, 0], y_t[:, 0]])) <= {1, -1}
    assert np.allclose(np.r_[xa, xa_t].mean(0), 0, atol=1e-9)        # standardised per column
    expect = np.where(which[rows] == 0, 1, -1)
    assert np.array_equal(np.r_[y[:, 0], y_t[:, 0]], expect)
    (a, b, c, y3), _ = NUS_WIDE_load_three_party_data(str(tmp_path), ["sky", "water", "person"])
    assert b.shape[1] == 3 and c.shape[1] == 3 and len(a) == len(y3) == int(0.8 * n)


def test_lending_club_two_and_three_party(tmp_path):
    """Lending Club VFL parties (reference data/lending_club_loan/lending_club_dataset.py:187-287) from a
    synthetic loan.csv with the dataset's columns: 2018 loans only, bad-loan target, standardised features,
    feature-group party split, 80/20 train/test, processed CSV cached."""
    import numpy as np
    from fedml_amd.data import lending_club as lc
    lc.write_synthetic_loan_csv(str(tmp_path / "loan.csv"), n=300)
    d = str(tmp_path) + "/"
    train, test = lc.loan_load_two_party_data(d)
    assert (tmp_path / "processed_loan.csv").exists()
    Xa, Xb, y = train
    n2018 = len(lc.prepare_data(str(tmp_path / "loan.csv")))
    assert Xa.shape == (int(0.8 * n2018), len(lc.QUALIFICATION + lc.LOAN))
    assert Xb.shape[1] == len(lc.DEBT + lc.REPAYMENT + lc.MULTI_ACC + lc.MAL_BEHAVIOR)
    assert y.shape == (Xa.shape[0], 1) and set(np.unique(y)) <= {0.0, 1.0} and not np.isnan(y).any()
    full = np.concatenate([Xa, test[0]])
    assert np.allclose(full.mean(0), 0, atol=1e-9) and np.allclose(full.std(0)[full.std(0) > 0], 1, atol=1e-9)
    tr3, te3 = lc.loan_load_three_party_data(d)
    assert len(tr3) == 4 and tr3[1].shape[1] == len(lc.DEBT + lc.REPAYMENT)
    assert tr3[2].shape[1] == len(lc.MULTI_ACC + lc.MAL_BEHAVIOR)
    assert np.allclose(tr3[0], Xa, rtol=1e-12, atol=1e-12)
