#!/bin/bash
# Bench-level A/B of tuning knobs: tools/bench_ab.sh "pair_cfg=1" "pair_cfg=0" ...
# prints ms/step and the per-stage MRF launch averages for each VO_TUNE setting
for c in "$@"; do
  VO_TUNE="$c" timeout -k 10 150 python bench.py --cpu-seconds 0 --steps 20 --no-configs > gpurun_out/b.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  python - "$c" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/b.json").read().strip().splitlines()[-1])
s = d["roofline"]["all_stages"]
print(sys.argv[1], d["ms_per_step"], {k: v["avg_ms"] for k, v in s.items()}, flush=True)
PY
done
