"""Lending Club loan data as vertical-FL parties (reference ``data/lending_club_loan/lending_club_dataset.py``,
``lending_club_feature_group.py``).

Pipeline (reference :148-202): read ``loan.csv`` → label each loan good / bad from ``loan_status`` → the
applicant's income (joint income when the joint verification status equals the individual one) → keep
loans issued in 2018 → map the categorical columns to integers → missing values −99 → standardise every
feature column (population std, as sklearn's StandardScaler) → cache ``processed_loan.csv``. The feature
columns are split into parties by the reference's feature groups: two parties = (qualification + loan) |
(debt + repayment + multi-account + delinquency), three parties = (qualification + loan) | (debt +
repayment) | (multi-account + delinquency). The first 80 % of the rows train, the rest test.

Differences from the reference, on purpose: the target column is attached by position (the reference's
``pd.concat(axis=1)`` aligns the re-indexed features with the filtered frame's original index, which
leaves NaN targets for every loan not issued in 2018's index range); a column whose std is 0 stays 0
instead of dividing by zero."""
import os
from typing import List

import numpy as np

QUALIFICATION = ["grade", "emp_length", "home_ownership", "annual_inc_comp", "verification_status",
                 "total_rev_hi_lim", "tot_hi_cred_lim", "total_bc_limit", "total_il_high_credit_limit"]
LOAN = ["loan_amnt", "term", "initial_list_status", "purpose", "application_type", "disbursement_method"]
DEBT = ["int_rate", "installment", "revol_bal", "revol_util", "out_prncp", "recoveries", "dti", "dti_joint",
        "tot_coll_amt", "mths_since_rcnt_il", "total_bal_il", "il_util", "max_bal_bc", "all_util", "bc_util",
        "total_bal_ex_mort", "revol_bal_joint", "mo_sin_old_il_acct", "mo_sin_old_rev_tl_op", "mo_sin_rcnt_rev_tl_op",
        "mort_acc", "num_rev_tl_bal_gt_0", "percent_bc_gt_75"]
REPAYMENT = ["num_sats", "num_bc_sats", "pct_tl_nvr_dlq", "bc_open_to_buy", "last_pymnt_amnt", "total_pymnt",
             "total_pymnt_inv", "total_rec_prncp", "total_rec_int", "total_rec_late_fee", "tot_cur_bal", "avg_cur_bal"]
MULTI_ACC = ["num_il_tl", "num_op_rev_tl", "num_rev_accts", "num_actv_rev_tl", "num_tl_op_past_12m", "open_rv_12m",
             "open_rv_24m", "open_acc_6m", "open_act_il", "open_il_12m", "open_il_24m", "total_acc", "inq_last_6mths",
             "open_acc", "inq_fi", "inq_last_12m", "acc_open_past_24mths"]
MAL_BEHAVIOR = ["num_tl_120dpd_2m", "num_tl_30dpd", "num_tl_90g_dpd_24m", "pub_rec_bankruptcies",
                "mths_since_recent_revol_delinq", "num_accts_ever_120_pd", "mths_since_recent_bc_dlq",
                "chargeoff_within_12_mths", "collections_12_mths_ex_med", "mths_since_last_major_derog",
                "acc_now_delinq", "pub_rec", "mths_since_last_delinq", "delinq_2yrs", "delinq_amnt", "tax_liens"]
ALL_FEATURES = QUALIFICATION + LOAN + DEBT + REPAYMENT + MULTI_ACC + MAL_BEHAVIOR

BAD_STATUS = {"Charged Off", "Default", "Does not meet the credit policy. Status:Charged Off", "In Grace Period",
              "Late (16-30 days)", "Late (31-120 days)"}
CATEGORICAL = {
    "grade": {"A": 6, "B": 5, "C": 4, "D": 3, "E": 2, "F": 1, "G": 0},
    "emp_length": {"< 1 year": 1, "1 year": 2, "2 years": 2, "3 years": 2, "4 years": 3, "5 years": 3,
                   "6 years": 3, "7 years": 4, "8 years": 4, "9 years": 4, "10+ years": 5},
    "home_ownership": {"RENT": 0, "MORTGAGE": 1, "OWN": 2, "ANY": 3, "NONE": 3, "OTHER": 3},
    "verification_status": {"Not Verified": 0, "Source Verified": 1, "Verified": 2},
    "term": {" 36 months": 0, " 60 months": 1},
    "initial_list_status": {"w": 0, "f": 1},
    "purpose": {"debt_consolidation": 0, "credit_card": 0, "small_business": 1, "educational": 2},  # else 3
    "application_type": {"Individual": 0, "Joint App": 1},
    "disbursement_method": {"Cash": 0, "DirectPay": 1},
}
_DEFAULT_CODE = {"purpose": 3, "emp_length": 0}   # the reference maps every other purpose to 3, NaN length to 0


def prepare_data(csv_path: str):
    """The 2018 loans of ``loan.csv`` with a 0/1 ``target`` (1 = bad loan), ``annual_inc_comp`` and the
    categorical columns mapped to integers (a pandas DataFrame)."""
    import pandas as pd
    df = pd.read_csv(csv_path, low_memory=False)
    df["target"] = df["loan_status"].isin(BAD_STATUS).astype(np.int64)
    joint = df["verification_status"] == df["verification_status_joint"]
    df["annual_inc_comp"] = np.where(joint, df["annual_inc_joint"], df["annual_inc"])
    df["issue_year"] = pd.to_datetime(df["issue_d"], format="mixed").dt.year
    for col, table in CATEGORICAL.items():
        if col in df:
            mapped = df[col].map(table)
            if col == "purpose":       # every purpose outside the table is class 3
                mapped = mapped.fillna(_DEFAULT_CODE[col])
            elif col == "emp_length":  # a missing employment length is class 0
                mapped = mapped.where(df[col].notna(), _DEFAULT_CODE[col])
            df[col] = mapped
    return df[df["issue_year"] == 2018].reset_index(drop=True)


def process_data(df):
    """Standardised feature matrix (missing → −99 first) with the target attached by position."""
    import pandas as pd
    X = df[ALL_FEATURES].apply(pd.to_numeric, errors="coerce").fillna(-99.0).to_numpy(np.float64)
    mu, sd = X.mean(0), X.std(0)
    X = (X - mu) / np.where(sd > 0, sd, 1.0)
    out = pd.DataFrame(X, columns=ALL_FEATURES)
    out["target"] = df["target"].to_numpy()
    return out


def load_processed_data(data_dir: str):
    import pandas as pd
    cached = os.path.join(data_dir, "processed_loan.csv")
    if os.path.exists(cached):
        return pd.read_csv(cached, low_memory=False)
    df = process_data(prepare_data(os.path.join(data_dir, "loan.csv")))
    df.to_csv(cached, index=False)
    return df


def _split(df, groups: List[List[str]]):
    parts = [df[g].to_numpy(np.float64) for g in groups]
    y = df["target"].to_numpy(np.float64).reshape(-1, 1)
    n = int(0.8 * len(y))
    return [p[:n] for p in parts] + [y[:n]], [p[n:] for p in parts] + [y[n:]]


def loan_load_two_party_data(data_dir: str):
    """([Xa_train, Xb_train, y_train], [Xa_test, Xb_test, y_test]); y is [n, 1]."""
    return _split(load_processed_data(data_dir), [QUALIFICATION + LOAN, DEBT + REPAYMENT + MULTI_ACC + MAL_BEHAVIOR])


def loan_load_three_party_data(data_dir: str):
    """([Xa, Xb, Xc, y] train, [Xa, Xb, Xc, y] test)."""
    return _split(load_processed_data(data_dir), [QUALIFICATION + LOAN, DEBT + REPAYMENT, MULTI_ACC + MAL_BEHAVIOR])


def write_synthetic_loan_csv(path: str, n: int = 200, seed: int = 0):
    """A ``loan.csv`` with the columns the pipeline reads (tests / offline demos; no download)."""
    import pandas as pd
    rng = np.random.default_rng(seed)
    cols = {}
    numeric = [c for c in ALL_FEATURES if c not in CATEGORICAL and c != "annual_inc_comp"]
    for c in numeric:
        v = rng.normal(50, 20, n)
        v[rng.random(n) < 0.05] = np.nan
        cols[c] = v
    for c, table in CATEGORICAL.items():
        keys = list(table) + (["wedding", "other"] if c == "purpose" else [])
        cols[c] = rng.choice(keys, n)
    cols["emp_length"] = np.where(rng.random(n) < 0.1, None, cols["emp_length"])
    cols["annual_inc"] = rng.normal(60000, 15000, n)
    cols["annual_inc_joint"] = rng.normal(90000, 20000, n)
    cols["verification_status_joint"] = rng.choice(list(CATEGORICAL["verification_status"]) + [None], n)
    cols["loan_status"] = rng.choice(["Fully Paid", "Current", "Charged Off", "Late (31-120 days)"], n)
    cols["issue_d"] = rng.choice(["Dec-2018", "Mar-2018", "Jun-2017"], n)
    pd.DataFrame(cols).to_csv(path, index=False)
