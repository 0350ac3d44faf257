#!/usr/bin/env python3
"""Dominant kernel and kernel families of the C4 / C5 training steps from serialized trace tail
stats (tools/trace_tail_stats.py) -> JSON read by bench.py (profiles/r04/train_dominant.json).
Family FLOPs per step (bench.train_step_flops' terms):
  C5: conv1d_kernel (forward + input gradients) 2 G + 7 D, wgrad kernels G + 2 D
      (G = generator forward, D = one MPD + MSD forward over the batch);
  C4: conv1d_kernel 2 x 719.9 GFLOP (the 771.4 GFLOP forward minus its 51.5 GFLOP of attention),
      wgrad kernels 719.9 GFLOP, attention forward + backward 5 x 51.5 GFLOP.
    python tools/train_dominant.py C4_TAIL.csv C5_TAIL.csv OUT.json"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

PEAK = bench.BF16_PEAK_TFLOPS


def load(path):
    return [dict(r, UsPerStep=float(r["UsPerStep"]), AvgUs=float(r["AvgUs"]), CallsPerStep=float(r["CallsPerStep"]))
            for r in csv.DictReader(open(path))]


def fam(rows, pred):
    return sum(r["UsPerStep"] for r in rows if pred(r["Name"]))


def reconcile(src):
    """The traced run's own clock: the tail's span per step (trace_tail_stats' JSON) and the bench line
    the profiled run printed (its ms_per_step, with the profiler attached)."""
    out = {}
    side = src.replace(".csv", ".json")
    if os.path.exists(side):
        out.update(json.load(open(side)))
    log = os.path.join(os.path.dirname(os.path.dirname(src)), os.path.basename(os.path.dirname(src)) + ".log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                try:
                    out["profiled_run_ms_per_step"] = json.loads(line)["ms_per_step"]
                except (ValueError, KeyError):
                    pass
    return out


def summary(rows, families, src):
    top = max(rows, key=lambda r: r["UsPerStep"])
    busy = sum(r["UsPerStep"] for r in rows)
    out = {"name": top["Name"], "avg_us": top["AvgUs"], "calls_per_step": top["CallsPerStep"],
           "share_of_step_kernel_time": round(top["UsPerStep"] / busy, 4), "kernel_us_per_step": round(busy, 1),
           "source": src, "families": {}}
    rec = reconcile(src)
    if rec:
        # shares are of the traced step's kernel time; the traced step (profiler attached: serialized
        # dispatches, per-dispatch overhead) is slower than the unprofiled bench line
        out["trace_clock"] = rec
        if rec.get("span_us_per_step"):
            out["kernel_busy_over_span"] = round(busy / rec["span_us_per_step"], 4)
    for label, (pred, flops) in families.items():
        us = fam(rows, pred)
        out["families"][label] = {"us_per_step": round(us, 1), "flops_per_step": flops,
                                  "tflops": round(flops / (us * 1e-6) / 1e12, 1) if us else None,
                                  "frac": round(flops / (us * 1e-6) / 1e12 / PEAK, 4) if us else None,
                                  "share_of_step_kernel_time": round(us / busy, 4)}
    return out


def main(c4, c5, out):
    G = bench.GEN_FLOPS_PER_SAMPLE * 16 * 8192
    D = bench.disc_forward_flops(8192, 16)
    conv = lambda n: "conv1d_kernel" in n  # noqa: E731
    wg = lambda n: "wgrad" in n  # noqa: E731
    att = lambda n: "attn" in n or "attention" in n  # noqa: E731
    res = {
        "train": summary(load(c4), {"conv1d_kernel (forward + input gradients)": (conv, 2 * 719.9e9),
                                    "wgrad kernels": (wg, 719.9e9),
                                    "attention forward + backward": (att, 5 * 51.5e9)}, os.path.relpath(c4)),
        "gan": summary(load(c5), {"conv1d_kernel (forward + input gradients)": (conv, 2 * G + 7 * D),
                                  "wgrad kernels": (wg, G + 2 * D)}, os.path.relpath(c5)),
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
