# software-pipelined pair kernels (pair_cfg 60: C = 128 SB; 34 / 35: C = 64 PIPE both / P1): parity, times
mkdir -p gpurun_out/r3k
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "(test_fused_resblock_pair_vs_torch_fp32 and (34- or 35- or 60-)) or (test_fused_resblock3_vs_torch_fp32 and (0- or 42- or 45-))" > gpurun_out/r3k/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3k/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/mrf_bench.py --stages 1 --tune pair_cfg=0,60 > gpurun_out/r3k/mrf_s1.txt 2>&1 || exit 1
timeout -k 10 200 python tools/mrf_bench.py --stages 2 --tune pair_cfg=0,34,35 > gpurun_out/r3k/mrf_s2.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r3k/mrf_s*.txt
