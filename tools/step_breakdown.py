#!/usr/bin/env python3
"""Per-kernel time of one steady-state bench step from a rocprofv3 kernel trace
(the launches between the last two conv_post dispatches).

    python tools/step_breakdown.py gpurun_out/prof_x/run_kernel_trace.csv [min_us]
"""
import csv
import sys
from collections import defaultdict


def main(path, min_us=0.0):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "conv_post" in r["Kernel_Name"]]
    step = rows[idx[-2] + 1: idx[-1] + 1]
    agg = defaultdict(lambda: [0, 0.0])
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        name = r["Kernel_Name"].split("(")[0][:80]
        agg[name][0] += 1
        agg[name][1] += d
    span = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
    busy = sum(v[1] for v in agg.values())
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        if t >= float(min_us):
            print(f"{t:9.1f} us  x{n:3d}  {name}")
    print(f"step span {span:.1f} us, kernels busy {busy:.1f} us ({100 * busy / span:.1f} %)")


if __name__ == "__main__":
    main(*sys.argv[1:])
