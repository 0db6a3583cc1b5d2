#!/usr/bin/env python3
"""Raw per-kernel counter dump of rocprofv3 PMC passes (each pass its own run with --kernel-trace).

usage: pmc_dump.py passdir1 [passdir2 ...]
Per kernel: calls, mean µs per call (first pass that has it), then every counter as its per-call mean, and
the ratios that stay meaningful whatever the counters' sampling scope is (both terms from the same pass):
  lds_wait% = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES     (wave-cycles spent waiting on LDS)
  valu%     = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES  lds_act% = SQ_ACTIVE_INST_LDS / SQ_WAVE_CYCLES
  wait_any% = SQ_WAIT_ANY / SQ_WAVE_CYCLES          ldsC%   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  occ       = SQ_WAVE_CYCLES / SQ_BUSY_CYCLES       (mean resident waves per SQ while busy)"""
import sys
from collections import defaultdict

sys.path.insert(0, __import__("os").path.dirname(__file__))
from pmc_table import load  # noqa: E402


def main():
    per = defaultdict(lambda: defaultdict(float))
    for d in sys.argv[1:]:
        dur, vals = load(d)
        calls = defaultdict(int)
        for did, (name, ns) in dur.items():
            calls[name] += 1
            per[name]["_ns@" + d] += ns
            for c, v in vals.get(did, {}).items():
                per[name][c + "@" + d] += v
        for name, n in calls.items():
            per[name]["_calls@" + d] = n
    for name, a in sorted(per.items(), key=lambda kv: -max(v for k, v in kv[1].items() if k.startswith("_ns@"))):
        passes = sorted({k.split("@", 1)[1] for k in a})
        d0 = passes[0]
        n0 = a["_calls@" + d0]
        print(f"{name}  calls {int(n0)}  {a['_ns@' + d0] / n0 / 1e3:.1f} us/call")
        ratios = []
        for d in passes:
            n = a.get("_calls@" + d, 1) or 1
            cs = {k.split("@")[0]: v / n for k, v in a.items() if k.endswith("@" + d) and not k.startswith("_")}
            print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(cs.items())))
            wc = cs.get("SQ_WAVE_CYCLES")
            for num, lab in (("SQ_WAIT_INST_LDS", "lds_wait%"), ("SQ_ACTIVE_INST_VALU", "valu%"),
                             ("SQ_ACTIVE_INST_LDS", "lds_act%"), ("SQ_WAIT_ANY", "wait_any%"),
                             ("SQ_WAIT_INST_ANY", "wait_inst%")):
                if wc and num in cs:
                    ratios.append(f"{lab}={100 * cs[num] / wc:.1f}")
            if cs.get("SQ_LDS_IDX_ACTIVE"):
                ratios.append(f"ldsC%={100 * cs.get('SQ_LDS_BANK_CONFLICT', 0) / cs['SQ_LDS_IDX_ACTIVE']:.1f}")
            if wc and cs.get("SQ_BUSY_CYCLES"):
                ratios.append(f"occ={wc / cs['SQ_BUSY_CYCLES']:.2f}")
        print("   -> " + "  ".join(ratios))


if __name__ == "__main__":
    main()
