# C = 32 wave-private kernels: parity (rb3_cfg 30/31, pair_cfg 50), then per-launch times
mkdir -p gpurun_out/r3f
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "(test_fused_resblock3_vs_torch_fp32 and (30- or 31- or 20-)) or (test_fused_resblock_pair_vs_torch_fp32 and -50])" > gpurun_out/r3f/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r3f/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/mrf_bench.py --stages 3 --tune rb3_cfg=0,30,31 --tune pair_cfg=0,50 > gpurun_out/r3f/mrf_bench.txt 2>&1; rc=$?; cat gpurun_out/r3f/mrf_bench.txt; exit $rc
