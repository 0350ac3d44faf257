# training tests after the FusedAdam version-bump fix; rb3 whole-conv weight groups (rb3_cfg 40/41)
mkdir -p gpurun_out/r3i
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_train_sizes.py tests/test_gpu_gan.py -q -m gpu --timeout 200 --timeout-method thread -k "optim or train_sizes or graphed or stft_loss or trainer" > gpurun_out/r3i/pytest_train.log 2>&1; rc=$?
tail -15 gpurun_out/r3i/pytest_train.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "test_fused_resblock3_vs_torch_fp32 and (40- or 41- or 0-)" > gpurun_out/r3i/pytest_rb3.log 2>&1; rc=$?; tail -3 gpurun_out/r3i/pytest_rb3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/mrf_bench.py --stages 2 --tune rb3_cfg=0,40,41 > gpurun_out/r3i/mrf_s2.txt 2>&1 || exit 1
grep block gpurun_out/r3i/mrf_s2.txt
