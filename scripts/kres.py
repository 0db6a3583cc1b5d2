#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: VGPR/AGPR, spills, LDS, occupancy
per kernel (filter with a substring). Usage: kres.py file.txt [substring]"""
import re
import sys

txt = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for b in re.split(r'remark: [^\n]*Function Name: ', txt)[1:]:
    name = b.split()[0]
    if flt not in name:
        continue

    def g(k):
        m = re.search(k + r': (\d+)', b)
        return int(m.group(1)) if m else -1
    occ = g(r'Occupancy \[waves/SIMD\]')
    lds = g(r'LDS Size \[bytes/block\]')
    print(f"{g('VGPRs'):4d}v {g('AGPRs'):4d}a spill {g('VGPRs Spill'):3d}/{g('SGPRs Spill'):3d} "
          f"occ {occ:2d} lds {lds:6d}  {name[:150]}")
