# training-side GPU tests (no -x: see every failure), then the default bench line
mkdir -p gpurun_out/r3h
timeout -k 10 700 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_train_sizes.py tests/test_gpu_train_glue.py tests/test_gpu_train.py tests/test_gpu_gan.py tests/test_gpu_ddp.py tests/test_checkpoint.py -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3h/pytest_train.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r3h/pytest_train.log | tail -60
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r3h/bench.json 2> gpurun_out/r3h/bench.err || exit 1
cat gpurun_out/r3h/bench.json
