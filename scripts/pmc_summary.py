"""Summarise a rocprofv3 --pmc counter_collection.csv: per kernel (first dispatch of each name by
default), the counters plus derived issue shares (quad-cycle SQ units)."""
import collections
import csv
import sys


def main(path, match=""):
    rows = list(csv.DictReader(open(path)))
    agg = collections.OrderedDict()
    for r in rows:
        k = r["Kernel_Name"]
        if match and match not in k:
            continue
        d = agg.setdefault((k, r["Dispatch_Id"]), {"_vgpr": r.get("VGPR_Count"), "_lds": r.get("LDS_Block_Size")})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    seen = set()
    for (k, did), d in agg.items():
        if k in seen:
            continue
        seen.add(k)
        name = k.split("(")[0][:90]
        out = [f"{name} #{did} vgpr={d.pop('_vgpr')} lds={d.pop('_lds')}"]
        wc = d.get("SQ_WAVE_CYCLES")
        for c, v in d.items():
            extra = f" ({100 * v / wc:.0f}% wave-cyc)" if wc and c.startswith("SQ_WAIT") or (wc and c == "SQ_ACTIVE_INST_ANY") else ""
            out.append(f"    {c:28s} {v:14.4g}{extra}")
        print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
