#!/bin/bash
# Bench-level A/B of environment settings: tools/bench_env_ab.sh "VO_RB3=0" "VO_RB3=1" ...
# prints ms/step and the per-stage MRF launch averages for each setting
for c in "$@"; do
  env $c timeout -k 10 150 python bench.py --cpu-seconds 0 --steps 20 --no-configs > gpurun_out/b.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  python - "$c" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/b.json").read().strip().splitlines()[-1])
s = d["roofline"]["all_stages"]
print(sys.argv[1], d["ms_per_step"], {k: (v["avg_ms"], v["launches"]) for k, v in s.items()}, flush=True)
PY
done
