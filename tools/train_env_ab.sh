#!/bin/bash
# C4 / C5 step A/B over environment settings (e.g. VO_LIB_PATH=abtmp/lib_old.so), interleaved twice:
# MODE=train|gan tools/train_env_ab.sh "" "VO_LIB_PATH=abtmp/lib_old.so"   ("" = defaults)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
for round in 1 2; do
  for c in "$@"; do
    env $c timeout -k 10 200 python bench.py --mode ${MODE:-train} --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/ab/e.out 2> gpurun_out/ab/e.err || { tail -5 gpurun_out/ab/e.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab/e.out').read().strip().splitlines()[-1]); print('round $round', repr(sys.argv[1]), d['ms_per_step'], flush=True)" "$c"
  done
done
