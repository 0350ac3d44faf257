#!/usr/bin/env python3
"""Summarize rocprofv3 --pmc CSVs per kernel (mean per dispatch)."""
import csv
import glob
import sys
from collections import defaultdict

d = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "conv1d" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("<")[1][:60]
        d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in d.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print("==", k)
    for c in sorted(m):
        print(f"   {c:28s} {m[c]:16.1f}")
    wc = m.get("SQ_WAVE_CYCLES", 0)
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_VMEM"):
            if c in m:
                print(f"   {c:28s} {100 * m[c] / wc:6.1f}% of wave cycles")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        print(f"   MFMA busy = {100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] * 1024):.1f}% (per SIMD, 1024 SIMDs)")
