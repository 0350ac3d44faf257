# round-3 GPU batch: training tests, then per-kernel SQ counters (tools/mrf_counters.sh)
mkdir -p gpurun_out/r3d
timeout -k 10 700 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_train_sizes.py tests/test_gpu_train_glue.py tests/test_gpu_train.py tests/test_gpu_gan.py tests/test_gpu_ddp.py tests/test_checkpoint.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3d/pytest_train.log 2>&1; rc=$?; tail -15 gpurun_out/r3d/pytest_train.log
for p in "pair 64 11 5" "pair 64 11 5 40" "rb3 64" "pair 32 7 3" "conv 256 3 1" "pair 128 11 5" "rb3 32"; do n=$(echo $p | tr " " _); bash tools/mrf_counters.sh gpurun_out/r3d/$n $p > gpurun_out/r3d/c_$n.txt 2>&1 || { echo FAIL $n; tail -5 gpurun_out/r3d/c_$n.txt; exit 1; }; rm -rf gpurun_out/r3d/$n; done
ls gpurun_out/r3d
exit $rc
