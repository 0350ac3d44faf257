#!/bin/bash
# C4 train-step A/B over VO_TUNE settings, interleaved twice: tools/train_tune_ab.sh "" "splitk_cfg=2" ...
# ("" = defaults); prints ms/step per setting and round
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
for round in 1 2; do
  for c in "$@"; do
    VO_TUNE="$c" timeout -k 10 200 python bench.py --mode ${MODE:-train} --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/ab/t.out 2> gpurun_out/ab/t.err || { tail -5 gpurun_out/ab/t.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab/t.out').read().strip().splitlines()[-1]); print('round $round', repr(sys.argv[1]), d['ms_per_step'], flush=True)" "$c"
  done
done
