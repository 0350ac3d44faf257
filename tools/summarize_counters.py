#!/usr/bin/env python3
"""Summarize rocprofv3 --pmc CSVs per kernel (mean per dispatch)."""
import csv
import glob
import sys
from collections import defaultdict

d = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if not any(s in r["Kernel_Name"] for s in ("conv1d", "pair", "rb3", "pb3", "rr3", "ups", "prw", "attn", "wgrad")):
            continue
        k = r["Kernel_Name"].split("(")[0][-80:]
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
        # GRBM_GUI_ACTIVE sums the 8 XCDs; MFMA busy cycles sum the 1024 SIMDs
        print(f"   MFMA busy = {100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (m['GRBM_GUI_ACTIVE'] / 8):.1f}% of SIMD cycles")
    if m.get("SQ_INSTS_MFMA", 0):
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
            if c in m:
                print(f"   {c:28s} {m[c] / m['SQ_INSTS_MFMA']:6.2f} per MFMA")
