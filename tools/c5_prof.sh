#!/bin/bash
# C5 (HiFi-GAN training) steady-state kernel breakdown: eager steps under rocprofv3 kernel trace,
# last 3 steps summarised by tools/trace_tail_stats.py (2 stft_mel launches per step).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5/prof -o run -- python bench.py --mode gan --steps 6 --warmup 2 --no-graph --cpu-seconds 0 > gpurun_out/c5/prof.log 2>&1 || exit 1
python tools/trace_tail_stats.py gpurun_out/c5/prof/run_kernel_trace.csv && rm -f gpurun_out/c5/prof/run_kernel_trace.csv
