#!/bin/bash
# Run GPU steps in order, each under its own time limit, stopping at the first step that faulted,
# aborted, crashed or timed out (exit 134 / 139 / 124 / 137 or > 128); a plain test failure (rc 1)
# does not stop the later steps.  Usage: tools/gpu_step.sh OUTDIR "cmd1" "cmd2" ...
OUT=$1; shift
mkdir -p "$OUT"
i=0
for cmd in "$@"; do
  i=$((i + 1))
  echo "== step $i: $cmd" | tee -a "$OUT/steps.log"
  timeout -k 10 ${STEP_TIMEOUT:-300} bash -c "$cmd" > "$OUT/step$i.log" 2>&1
  rc=$?
  echo "== step $i rc=$rc" | tee -a "$OUT/steps.log"
  tail -${TAIL:-15} "$OUT/step$i.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
