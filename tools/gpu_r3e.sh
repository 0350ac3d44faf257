# rb3 VALU-diet check: parity of every rb3 config, then per-launch times (rb3_cfg 20 = round-2 epilogues)
mkdir -p gpurun_out/r3e
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q --timeout 200 --timeout-method thread -k "resblock3 or rb3 or mrf or generator" > gpurun_out/r3e/pytest_rb3.log 2>&1; rc=$?; tail -5 gpurun_out/r3e/pytest_rb3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/mrf_bench.py --stages 1,2,3 --tune rb3_cfg=20,0 > gpurun_out/r3e/mrf_bench.txt 2>&1; rc=$?; grep block gpurun_out/r3e/mrf_bench.txt; exit $rc
