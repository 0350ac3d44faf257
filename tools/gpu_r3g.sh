# VALU-diet pair kernels: parity (pair_cfg 0 = VD defaults, 8 / 33 = round-2 kernels), then per-launch times
mkdir -p gpurun_out/r3g
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "test_fused_resblock_pair_vs_torch_fp32 or test_fused_resblock3_vs_torch_fp32" > gpurun_out/r3g/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r3g/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/mrf_bench.py --stages 1 --tune pair_cfg=8,0 > gpurun_out/r3g/mrf_s1.txt 2>&1 || exit 1
timeout -k 10 200 python tools/mrf_bench.py --stages 2 --tune pair_cfg=33,0 > gpurun_out/r3g/mrf_s2.txt 2>&1 || exit 1
timeout -k 10 200 python tools/mrf_bench.py --stages 3 --tune pair_cfg=8,0,50 > gpurun_out/r3g/mrf_s3.txt 2>&1 || exit 1
cat gpurun_out/r3g/mrf_s*.txt | grep -v amdgpu.ids
