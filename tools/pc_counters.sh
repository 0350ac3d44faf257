#!/bin/bash
# Counters of the C = 128 k = 11 d = 5 pair: round-3 kernel (pair_cfg 70), round-4 producer-role
# kernel (pc_cfg 0) and its no-DMA ablation (pc_cfg 10, ablation library).  Run on the GPU box.
OUT=${1:-gpurun_out/pc_counters}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tools/mrf_counters.sh $OUT/r3 pair 128 11 5 70 || exit 1
tools/mrf_counters.sh $OUT/pc pair 128 11 5 || exit 1
VO_LIB_PATH=visual_onoma_to_wave_amd/lib/libvonoma_abl.so VO_TUNE=pc_cfg=10 tools/mrf_counters.sh $OUT/pc_noload pair 128 11 5 || exit 1
