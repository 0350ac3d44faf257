#!/bin/bash
# HBM traffic per MRF launch: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; each in its
# own run, counters only) over a short bench, summarised by tools/pmc_traffic.py.
# Usage: tools/pmc_round.sh TAG   -> gpurun_out/TAG/pmc/{fetch_size,write_size}.csv, traffic.json
set -o pipefail
TAG=${1:-pmc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG/pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | tr 'A-Z' 'a-z')
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/raw_$lc" -o run -- python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-configs > "$OUT/$lc.log" 2>&1 || { tail -5 "$OUT/$lc.log"; exit 1; }
  f=$(find "$OUT/raw_$lc" -name '*counter_collection.csv' | head -1)
  [ -n "$f" ] || { echo "no counter csv for $c"; exit 1; }
  python - "$f" "$OUT/$lc.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
keep = ["Kernel_Name", "Counter_Name", "Counter_Value"]
with open(sys.argv[2], "w", newline="") as f:
    w = csv.DictWriter(f, keep)
    w.writeheader()
    for r in rows:
        if any(k in r["Kernel_Name"] for k in ("mrf_", "conv1d_kernel", "ups_kernel", "upsw_kernel", "conv_post_rows")):
            w.writerow({k: r[k] for k in keep})
PY
  rm -rf "$OUT/raw_$lc"
done
python tools/pmc_traffic.py "$OUT/fetch_size.csv" "$OUT/write_size.csv" "$OUT/traffic.json" && cat "$OUT/traffic.json"
