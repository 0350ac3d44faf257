set -o pipefail
mkdir -p gpurun_out/ab
for i in 1 2; do
for c in 0 2 1; do
  VO_TUNE=splitk_cfg=$c timeout -k 10 200 python bench.py --steps 20 --cpu-seconds 0 --no-kernel-timer > gpurun_out/ab/b_${c}_$i.out 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab/b_${c}_$i.out').read().strip().splitlines()[-1]); print('splitk_cfg=$c', d['ms_per_step'])"
done; done
