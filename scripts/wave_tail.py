#!/usr/bin/env python3
"""Grid fill of every kernel in a rocprofv3 kernel trace (csv): workgroups per dispatch, resident workgroups per CU
(from the dispatch's VGPR / AGPR / LDS / wave counts, MI355X: 256 CUs, 4 SIMDs of 512 registers per lane, 160 KiB
LDS, ≤ 32 waves per CU), the number of workgroup waves and the tail efficiency = waves / ⌈waves⌉ (the share of the
last wave's slots that hold work when every workgroup takes the same time).

    python scripts/wave_tail.py gpurun_out/r5b/p13/.../run_kernel_trace.csv [--top 30] [--skip-frac 0.5]
"""
import argparse
import collections
import csv
import math

CUS, SIMD_REGS, LDS, MAX_WAVES = 256, 512, 160 * 1024, 32


def col(r, *names, default=0):
    for n in names:
        if n in r and r[n] not in ("", None):
            return r[n]
    return default


def occupancy(wg_threads, vgpr, agpr, lds):
    waves = max(1, math.ceil(wg_threads / 64))
    regs = vgpr + agpr
    alloc = max(8, math.ceil(max(regs, 1) / 8) * 8)
    per_simd = min(8, SIMD_REGS // alloc)
    by_regs = (4 * per_simd) // waves          # waves of one workgroup spread over the 4 SIMDs
    by_lds = LDS // lds if lds else 64
    by_waves = MAX_WAVES // waves
    return max(1, min(by_regs, by_lds, by_waves))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--skip-frac", type=float, default=0.5)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(col(r, "Start_Timestamp")))
    rows = rows[int(len(rows) * a.skip_frac):]
    agg = collections.defaultdict(lambda: [0, 0.0, None])
    for r in rows:
        name = col(r, "Kernel_Name", "KernelName")
        if "Grid_Size_X" in r:     # rocprofv3: 3-D grid and workgroup in work-items
            grid = math.prod(int(col(r, "Grid_Size_" + d, default=1) or 1) for d in "XYZ")
            wg = math.prod(int(col(r, "Workgroup_Size_" + d, default=1) or 1) for d in "XYZ")
        else:
            grid = int(col(r, "Grid_Size", default=0) or 0)
            wg = int(col(r, "Workgroup_Size", default=256) or 256)
        vgpr = int(col(r, "VGPR_Count", "Arch_VGPR_Count", default=0) or 0)
        agpr = int(col(r, "Accum_VGPR_Count", default=0) or 0)
        lds = int(col(r, "LDS_Block_Size", "Lds_Size", "LDS_Size", default=0) or 0)
        dur = (int(col(r, "End_Timestamp")) - int(col(r, "Start_Timestamp"))) / 1e3
        nwg = max(1, grid // max(1, wg))
        key = (name[:90], nwg, wg, vgpr, agpr, lds)
        e = agg[key]
        e[0] += 1
        e[1] += dur
    tot = sum(v[1] for v in agg.values())
    print(f"{'us total':>9} {'calls':>5} {'us/call':>8} {'WGs':>6} {'thr':>4} {'vgpr':>4} {'agpr':>4} {'lds':>6} "
          f"{'WG/CU':>5} {'waves':>6} {'tail%':>5}  kernel")
    for (name, nwg, wg, vgpr, agpr, lds), (n, us, _) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        occ = occupancy(wg, vgpr, agpr, lds)
        waves = nwg / (CUS * occ)
        tail = 100.0 * waves / math.ceil(waves)
        print(f"{us:9.0f} {n:5d} {us / n:8.1f} {nwg:6d} {wg:4d} {vgpr:4d} {agpr:4d} {lds:6d} {occ:5d} {waves:6.2f} "
              f"{tail:5.0f}  {name}")
    print(f"total {tot:.0f} us over {sum(v[0] for v in agg.values())} dispatches")


if __name__ == "__main__":
    main()
