#!/bin/bash
# batched weight norm: the full GPU suite, then the C5 bench with and without it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for c in VO_BATCHED_WN=0 VO_BATCHED_WN=1 VO_BATCHED_WN=0 VO_BATCHED_WN=1; do
  env $c timeout -k 10 200 python bench.py --mode gan --cpu-seconds 0 > gpurun_out/gan.json 2> gpurun_out/gan.err || { tail -20 gpurun_out/gan.err; exit 1; }
  echo $c; tail -1 gpurun_out/gan.json | cut -c1-200
done
