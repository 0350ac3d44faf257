# software-pipelined rb3 tap loops (rb3_cfg 42-44): parity, then per-launch times
mkdir -p gpurun_out/r3j
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "test_fused_resblock3_vs_torch_fp32 and (42- or 43- or 44-)" > gpurun_out/r3j/pytest_rb3.log 2>&1; rc=$?; tail -3 gpurun_out/r3j/pytest_rb3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/mrf_bench.py --stages 1 --tune rb3_cfg=0,42 > gpurun_out/r3j/mrf_s1.txt 2>&1 || exit 1
timeout -k 10 200 python tools/mrf_bench.py --stages 2 --tune rb3_cfg=0,42,43,44,40 > gpurun_out/r3j/mrf_s2.txt 2>&1 || exit 1
grep block gpurun_out/r3j/mrf_s*.txt
