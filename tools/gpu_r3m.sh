# C2 (acoustic model) kernel sequence of one step, serialized trace
mkdir -p gpurun_out/r3m
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3m/c2 -o run -- python bench.py --mode c2 --steps 3 --warmup 2 --cpu-seconds 0 > gpurun_out/r3m/c2.out 2>&1 || { tail -20 gpurun_out/r3m/c2.out; exit 1; }
f=$(find gpurun_out/r3m/c2 -name '*kernel_trace.csv' | head -1)
python tools/trace_sequence.py "$f" vfe_kernel > gpurun_out/r3m/c2_sequence.txt || exit 1
rm -rf gpurun_out/r3m/c2
tail -45 gpurun_out/r3m/c2_sequence.txt
