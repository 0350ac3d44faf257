#!/bin/bash
# usage: tools/wgrad_counters.sh OUTDIR (GPU box): the two PMC passes of tools/mrf_counters.sh over
# tools/probes/wgrad_probe.py, then the per-kernel summary
out=$1
mkdir -p $out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $out/p$i -o run -- python tools/probes/wgrad_probe.py > $out/p$i.log 2>&1 || exit 1
done
python tools/summarize_counters.py $out
