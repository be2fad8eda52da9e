#!/bin/bash
# GPU step: bk_conv3x3 timing + PMC counters (one counter group per pass, kernel-trace only).
# usage: tools/gpu/convpmc.sh [batch]
set -o pipefail
B=${1:-256}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/convpmc
timeout -k 10 120 python tools/conv_bench.py 200 64 $B > gpurun_out/convpmc/bench.json 2> gpurun_out/convpmc/bench.err || exit 1
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_BUSY_CYCLES SQ_WAVES" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" "SQ_INSTS_MFMA SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/convpmc/p$i -o c --output-format csv -- python tools/conv_bench.py 20 64 $B > gpurun_out/convpmc/p$i.log 2>&1 || exit 1
done
