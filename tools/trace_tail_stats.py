#!/usr/bin/env python3
"""Steady-state per-kernel time from a rocprofv3 kernel trace: only the dispatches after the
N-th-from-last occurrence of a marker kernel (default: the last 3 GAN steps, 2 stft_mel
dispatches per step), so one-off work (MIOpen Find, warm-up) is excluded.  Writes a compact
CSV next to the trace (safe to copy back: the full trace can exceed gpurun's 64 MiB).

    python tools/trace_tail_stats.py TRACE.csv [marker=stft_mel_kernel] [occurrences=6] [steps=3]
"""
import csv
import sys
from collections import defaultdict


def main(path, marker="stft_mel_kernel", occ=6, steps=3):
    occ, steps = int(occ), int(steps)
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    if marker.startswith("FRACTION:"):  # the last fraction of all dispatches (steady-state steps)
        start = int(len(rows) * (1.0 - float(marker.split(":")[1])))
    else:
        idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
        start = idx[-occ] if len(idx) >= occ else 0
    tail = rows[start:]
    agg = defaultdict(lambda: [0, 0.0])
    for r in tail:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        agg[r["Kernel_Name"][:160]][0] += 1
        agg[r["Kernel_Name"][:160]][1] += d
    span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
    busy = sum(v[1] for v in agg.values())
    out = path.replace(".csv", "_tail_stats.csv")
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "CallsPerStep", "UsPerStep", "AvgUs", "Percent"])
        for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([name, round(n / steps, 2), round(t / steps, 2), round(t / n, 3), round(100 * t / busy, 2)])
    print(f"{len(tail)} dispatches over {steps} steps: span {span / steps:.1f} us/step, kernels busy "
          f"{busy / steps:.1f} us/step -> {out}")
    import json
    with open(out.replace(".csv", ".json"), "w") as f:  # the tail's own clock, for reconciliation
        json.dump({"steps": steps, "dispatches": len(tail), "span_us_per_step": round(span / steps, 1),
                   "kernels_busy_us_per_step": round(busy / steps, 1)}, f, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
