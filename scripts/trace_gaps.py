#!/usr/bin/env python3
"""Device idle time between kernels from a rocprofv3 kernel trace (csv): for the busiest stretch of the run
(kernels after the first `--skip-ms` of GPU activity), the union of kernel intervals vs the wall span, the
gap histogram, and the kernels that most often follow a long gap.

    python scripts/trace_gaps.py gpurun_out/prof_c13b/.../c13_kernel_trace.csv [--skip-ms 0]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--skip-frac", type=float, default=0.5, help="ignore the first fraction of kernels (warm-up)")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    rows = rows[int(len(rows) * a.skip_frac):]
    busy, gaps, last_end = 0, [], None
    after = collections.Counter()
    cur_s, cur_e = rows[0][0], rows[0][1]
    for s, e, name in rows:
        if last_end is not None and s > last_end:
            gaps.append(s - last_end)
            if s - last_end > 20000:
                after[name[:80]] += 1
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        last_end = max(last_end or 0, e)
    busy += cur_e - cur_s
    span = rows[-1][1] - rows[0][0]
    print(f"kernels {len(rows)}  span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f} %)  "
          f"idle {(span - busy) / 1e6:.2f} ms")
    small = [g for g in gaps if g <= 20000]
    big = [g for g in gaps if g > 20000]
    print(f"gaps ≤ 20 µs: {len(small)} totalling {sum(small) / 1e6:.2f} ms (mean {sum(small) / max(1, len(small)) / 1e3:.1f} µs)")
    print(f"gaps > 20 µs: {len(big)} totalling {sum(big) / 1e6:.2f} ms")
    for name, n in after.most_common(10):
        print(f"  {n:5d}  after a > 20 µs gap: {name}")


if __name__ == "__main__":
    main()
