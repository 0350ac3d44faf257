#!/usr/bin/env python3
"""Per-launch HBM traffic of the MRF kernels (and the streaming upsamplers / conv_post) from
two rocprofv3 --pmc passes.

FETCH_SIZE and WRITE_SIZE are collected in separate passes (they do not fit one TCC
pass).  Per MI355X_MICROARCH.md section HBM: both are KB; on gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced streaming read, so it is doubled.  Result:
{"mrf_s<i>": {"hbm_bytes_per_launch", "fetch_bytes", "write_bytes", "launches"}}.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv OUT.json [FETCH2.csv WRITE2.csv ...]
"""
import csv
import json
import re
import sys
from collections import defaultdict

PAIR_STAGE = {256: "mrf_s0", 128: "mrf_s1", 64: "mrf_s2", 32: "mrf_s3"}


def load(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        if name.startswith("dec_ffn_w1 "):  # tools/conv_probe.py dec_ffn_w1 (the C2 dominant conv alone)
            acc["dec_ffn_w1"].append(float(r["Counter_Value"]))
            continue
        m = re.search(r"conv1d_kernel<[^>]*?(?:true|false),\s*(\d+)", name)  # ROLE follows the NICE flag
        if m and m.group(1) != "0":
            acc[f"mrf_s{int(m.group(1)) - 1}"].append(float(r["Counter_Value"]))
            continue
        m = re.search(r"mrf_(?:pair2?|rb3|rr3w?|rrp|prw)_kernel<(\d+),", name)  # fused pairs / blocks: stage by width
        if m and int(m.group(1)) in PAIR_STAGE:
            acc[PAIR_STAGE[int(m.group(1))]].append(float(r["Counter_Value"]))
            continue
        m = re.search(r"ups(w?)_kernel<(\d+),", name)  # streaming upsamplers: by input width
        if m:
            acc[{"128": "ups2", "64": "ups3", "256": "ups1"}.get(m.group(2), "ups_ci" + m.group(2))].append(
                float(r["Counter_Value"]))
            continue
        if "conv_post_rows_kernel" in name:
            acc["conv_post"].append(float(r["Counter_Value"]))
    return acc


def main(fetch_csv, write_csv, out, *extra):
    f = load(fetch_csv, "FETCH_SIZE")
    w = load(write_csv, "WRITE_SIZE")
    for fx, wx in zip(extra[0::2], extra[1::2]):  # further (FETCH, WRITE) csv pairs, e.g. the C2 probe
        for k, v in load(fx, "FETCH_SIZE").items():
            f[k] += v
        for k, v in load(wx, "WRITE_SIZE").items():
            w[k] += v
    res = {}
    for tag in sorted(set(f) | set(w)):
        fb = 2.0 * 1024 * sum(f[tag]) / max(1, len(f[tag]))
        wb = 1024 * sum(w[tag]) / max(1, len(w[tag]))
        res[tag] = {"hbm_bytes_per_launch": fb + wb, "fetch_bytes": fb, "write_bytes": wb,
                    "launches": len(f[tag]),
                    "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KB -> bytes"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
