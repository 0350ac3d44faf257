#!/bin/bash
# Round profile set (rounds 3-4): a SERIALIZED rocprofv3 kernel trace of the bench step (no acoustic /
# vocoder pipeline, the C = 256 MRF chains one after another -- the configuration of bench.py's
# roofline pass), its steady-state tail stats, and the HBM traffic per launch from separate
# FETCH_SIZE / WRITE_SIZE --pmc passes over the same command (+ the C2 decoder FFN w_1 conv alone).
# Usage: tools/prof_round.sh TAG   -> gpurun_out/TAG/{trace,pmc}
set -o pipefail
TAG=${1:-prof}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT/pmc"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export VO_MRF_STREAMS=0
BENCH="python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-configs --no-pipeline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $BENCH > "$OUT/trace_bench.out" 2>&1 || { tail -20 "$OUT/trace_bench.out"; exit 1; }
python tools/trace_tail_stats.py "$OUT/trace/run_kernel_trace.csv" conv_post_rows_kernel 4 3 || exit 1
rm -f "$OUT/trace/run_kernel_trace.csv"
PMCB="python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-configs --no-pipeline"
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | tr 'A-Z' 'a-z')
  for what in bench c2; do
    if [ $what = bench ]; then CMD=$PMCB; else CMD="python tools/conv_probe.py dec_ffn_w1"; fi
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc/raw_${what}_$lc" -o run -- $CMD > "$OUT/pmc/${what}_$lc.log" 2>&1 || { tail -5 "$OUT/pmc/${what}_$lc.log"; exit 1; }
    f=$(find "$OUT/pmc/raw_${what}_$lc" -name '*counter_collection.csv' | head -1)
    [ -n "$f" ] || { echo "no counter csv for $c $what"; exit 1; }
    python - "$f" "$OUT/pmc/${what}_$lc.csv" $what <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
keep = ["Kernel_Name", "Counter_Name", "Counter_Value"]
with open(sys.argv[2], "w", newline="") as f:
    w = csv.DictWriter(f, keep)
    w.writeheader()
    for r in rows:
        n = r["Kernel_Name"]
        if sys.argv[3] == "c2":
            if "conv1d_kernel" in n:
                w.writerow({"Kernel_Name": "dec_ffn_w1 " + n, "Counter_Name": r["Counter_Name"],
                            "Counter_Value": r["Counter_Value"]})
        elif any(k in n for k in ("mrf_", "conv1d_kernel", "ups_kernel", "upsw_kernel", "conv_post_rows")):
            w.writerow({k: r[k] for k in keep})
PY
    rm -rf "$OUT/pmc/raw_${what}_$lc"
  done
done
python tools/pmc_traffic.py "$OUT/pmc/bench_fetch_size.csv" "$OUT/pmc/bench_write_size.csv" "$OUT/pmc/traffic.json" \
    "$OUT/pmc/c2_fetch_size.csv" "$OUT/pmc/c2_write_size.csv"
