#!/bin/bash
# rocprofv3 kernel stats of the C2 line alone (acoustic model, B = 32, T_mel = 512)
set -o pipefail
OUT=gpurun_out/c2prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python bench.py --mode c2 --steps 10 --cpu-seconds 0 > $OUT/bench.out 2>&1 || { tail -20 $OUT/bench.out; exit 1; }
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/c2prof/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total ms", tot / 1e6)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:150]}')
PY
rm -f $OUT/run_kernel_trace.csv
