#!/bin/bash
# A/B of the concurrent conv-path MRF chains: the new tests, the bench step and the C3 line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mrf_streams.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mrfs_pytest.log 2>&1 || { tail -30 gpurun_out/mrfs_pytest.log; exit 1; }
tail -2 gpurun_out/mrfs_pytest.log
bash tools/bench_env_ab.sh "VO_MRF_STREAMS=0" "VO_MRF_STREAMS=1" "VO_MRF_STREAMS=0" "VO_MRF_STREAMS=1" || exit 1
for c in VO_MRF_STREAMS=0 VO_MRF_STREAMS=1; do
  env $c timeout -k 10 150 python bench.py --mode c3 --cpu-seconds 0 --steps 10 > gpurun_out/c3.json 2> gpurun_out/c3.err || { tail -5 gpurun_out/c3.err; exit 1; }
  python -c "
import json,sys; d=json.loads(open('gpurun_out/c3.json').read().strip().splitlines()[-1])
print(sys.argv[1], d['ms_per_step'], {k:(v['avg_ms'],v['launches']) for k,v in d['roofline']['all_stages'].items()})" "$c"
done
