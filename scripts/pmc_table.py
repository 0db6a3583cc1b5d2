#!/usr/bin/env python3
"""Per-kernel roofline table from rocprofv3 PMC passes (each pass its own run with --kernel-trace).

usage: pmc_table.py out.txt passdir1 [passdir2 ...]
Joins every pass's counter_collection.csv with its kernel_trace.csv on the dispatch id and reports per
kernel (full template name, shortened): calls, GPU ms (from the trace of the first pass that has the
kernel), HBM read GB (2 x FETCH_SIZE: on gfx950 FETCH_SIZE tallies half the bytes of 16-B-per-lane streaming
reads, MI355X_MICROARCH.md 'HBM'), write GB (WRITE_SIZE), achieved TB/s = (read + write) / time, and
MFMA-busy % = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel time x 2.4 GHz). SQ_VALU_MFMA_BUSY_CYCLES is the
chip-wide sum of matrix-pipe busy cycles (checked: a 30.2-GFLOP fp32 3x3 layer reports 4.72e8 = its 14.7 M
v_mfma_f32_16x16x4_f32 x 32 cycles, whatever the kernel's duration), so the ratio is the fraction of all
SIMD-cycles the matrix pipes were busy, <= 100 %. LDS bank-conflict % = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.
(GRBM_GUI_ACTIVE is not used: its per-dispatch value does not track the kernel's duration on this pool.)"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(n):
    n = n.replace("prec::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    return n[:70]


def load(d):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    dur = {}
    for f in kt:
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = (short(r["Kernel_Name"]), float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    vals = defaultdict(lambda: defaultdict(float))
    for f in cc:
        for r in csv.DictReader(open(f)):
            vals[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    return dur, vals


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    agg = defaultdict(lambda: defaultdict(float))
    for d in dirs:
        dur, vals = load(d)
        seen = defaultdict(float)
        for did, (name, ns) in dur.items():
            seen[name] += ns
            vd = vals.get(did, {})
            for c, v in vd.items():
                if c == "GRBM_GUI_ACTIVE":   # kept per pass: the MFMA ratio uses its own pass's cycles
                    c = "GRBM_GUI_ACTIVE_mfma" if "SQ_VALU_MFMA_BUSY_CYCLES" in vd else "GRBM_GUI_ACTIVE@" + d
                agg[name][c] += v
            agg[name]["_calls_" + d] += 1
        for name, ns in seen.items():
            if "_ns" not in agg[name]:
                agg[name]["_ns"] = ns
                agg[name]["_calls"] = agg[name]["_calls_" + d]
    rows = sorted(agg.items(), key=lambda kv: -kv[1].get("_ns", 0))
    tot = sum(a.get("_ns", 0) for _, a in rows)
    lines = [f"{'kernel':70s} {'calls':>6s} {'ms':>8s} {'%':>5s} {'rd_GB':>7s} {'wr_GB':>7s} {'TB/s':>6s} "
             f"{'mfma%':>6s} {'ldsC%':>6s}"]
    for name, a in rows[:40]:
        ms = a.get("_ns", 0) / 1e6
        rd = 2 * a.get("FETCH_SIZE", float("nan")) * 1024 / 1e9
        wr = a.get("WRITE_SIZE", float("nan")) * 1024 / 1e9
        tbs = (rd + (wr if wr == wr else 0)) / (ms / 1e3) / 1e3 if ms > 0 and rd == rd else float("nan")
        mf = a.get("SQ_VALU_MFMA_BUSY_CYCLES")
        mfp = 100 * mf / (1024 * ms * 1e-3 * 2.4e9) if mf is not None and ms > 0 else float("nan")
        lc, la = a.get("SQ_LDS_BANK_CONFLICT"), a.get("SQ_LDS_IDX_ACTIVE")
        lcp = 100 * lc / la if lc is not None and la else float("nan")
        lines.append(f"{name:70s} {int(a.get('_calls', 0)):6d} {ms:8.1f} {100 * ms * 1e6 / tot:5.1f} {rd:7.2f} "
                     f"{wr:7.2f} {tbs:6.2f} {mfp:6.1f} {lcp:6.1f}")
    lines.append(f"total kernel time {tot / 1e6:.1f} ms")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:45]))


if __name__ == "__main__":
    main()
