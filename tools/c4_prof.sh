set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/c4
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/c4/bench_train.out 2>&1 || exit 1
tail -1 gpurun_out/c4/bench_train.out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4/prof -o run -- python bench.py --mode train --steps 10 --warmup 3 --no-graph --cpu-seconds 0 > gpurun_out/c4/prof.log 2>&1 || exit 1
python tools/trace_tail_stats.py gpurun_out/c4/prof/run_kernel_trace.csv FRACTION:0.5 5 5 && rm -f gpurun_out/c4/prof/run_kernel_trace.csv
