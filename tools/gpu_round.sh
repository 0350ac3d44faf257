#!/bin/bash
# One GPU pass: GPU tests, the default bench line, and a rocprofv3 kernel-trace summary of the
# same bench command (steady-state tail + whole-run stats).  Usage: tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python bench.py > "$OUT/bench.out" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
tail -1 "$OUT/bench.out" > "$OUT/bench.json"
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 10 --cpu-seconds 0 --no-configs > /dev/null 2>&1 || exit 1
python tools/trace_tail_stats.py "$OUT/prof/run_kernel_trace.csv" conv_post_rows_kernel 4 3 && rm -f "$OUT/prof/run_kernel_trace.csv"
