"""Print the kernel sequence of the last step of a rocprofv3 --kernel-trace CSV (names shortened,
durations in us, gaps between consecutive kernels), plus per-name totals over that step.
Usage: python tools/trace_sequence.py run_kernel_trace.csv FIRST_KERNEL_SUBSTRING [steps]
A step starts at each occurrence of FIRST_KERNEL_SUBSTRING; the last complete one is printed."""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(.*$", "", n)
    n = n.replace("void ", "").replace("vo::", "")
    return n[:90]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marker = sys.argv[2]
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(starts) < 2:
        print("fewer than two steps found")
        return
    a, b = starts[-2], starts[-1]
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    prev_end = t0
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = (e - s) / 1e3
        print(f"{(s - t0) / 1e3:9.1f} {d:8.1f} gap {(s - prev_end) / 1e3:6.1f}  {short(r['Kernel_Name'])}")
        prev_end = max(prev_end, e)
        tot[short(r["Kernel_Name"])] += d
        cnt[short(r["Kernel_Name"])] += 1
    span = (int(step[-1]["End_Timestamp"]) - t0) / 1e3
    print(f"step span {span:.1f} us, kernel sum {sum(tot.values()):.1f} us, {len(step)} kernels")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{v:9.1f} us {cnt[k]:4d}x  {k}")


if __name__ == "__main__":
    main()
