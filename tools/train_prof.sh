#!/bin/bash
# Serialized kernel traces of the graphed C4 / C5 training steps (the bench's single-GPU configs):
# rocprofv3 --kernel-trace --stats over `bench.py --mode train|gan`, the last 3 steps summarised by
# tools/trace_tail_stats.py (marker: the optimizer's step-count increment, once per param group and
# step -- C4 1 / step at its end, C5 2 / step: D's mid-step, G's at the end -- so the tail starts at
# the (3 x per-step + 1)-th last one: the end of step N - 3), then tools/train_dominant.py ->
# OUT/train_dominant.json.
# Usage (GPU box): tools/train_prof.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/train_prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4" -o run -- python bench.py --mode train --steps 8 --warmup 3 > "$OUT/c4.log" 2>&1 || { tail "$OUT/c4.log"; exit 1; }
python tools/trace_tail_stats.py "$OUT/c4/run_kernel_trace.csv" opt_step_increment 4 3 && rm -f "$OUT/c4/run_kernel_trace.csv" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5" -o run -- python bench.py --mode gan --steps 8 --warmup 3 > "$OUT/c5.log" 2>&1 || { tail "$OUT/c5.log"; exit 1; }
python tools/trace_tail_stats.py "$OUT/c5/run_kernel_trace.csv" opt_step_increment 7 3 && rm -f "$OUT/c5/run_kernel_trace.csv" || exit 1
python tools/train_dominant.py "$OUT/c4/run_kernel_trace_tail_stats.csv" "$OUT/c5/run_kernel_trace_tail_stats.csv" "$OUT/train_dominant.json"
