#!/bin/bash
# Bench-level A/B of two builds of libvonoma.so, interleaved (A B A B ...) on one box:
# tools/bench_libs.sh A.so B.so [rounds] -> ms/step and the MRF stage averages per run
a=$1; b=$2; n=${3:-2}
for i in $(seq "$n"); do
  for lib in "$a" "$b"; do
    VO_LIB_PATH=$lib timeout -k 10 150 python bench.py --cpu-seconds 0 --steps 30 --no-configs > gpurun_out/bl.json 2> gpurun_out/bl.err || { tail -5 gpurun_out/bl.err; exit 1; }
    python - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/bl.json").read().strip().splitlines()[-1])
s = d["roofline"]["all_stages"]
print(sys.argv[1].split("/")[-1], d["ms_per_step"], {k: round(v["avg_ms"], 4) for k, v in s.items()}, flush=True)
PY
  done
done
