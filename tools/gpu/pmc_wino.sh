#!/bin/bash
# GPU step: stall counters of bk_conv3x3 (Winograd form at even N) at B=1024, one counter group per
# pass, kernel-trace only; optional $1 = library path (BK_LIB).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
[ -n "$1" ] && export BK_LIB=$1
out=gpurun_out/pmc_wino
mkdir -p $out
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU" "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --kernel-trace -d $out/p$i -o c --output-format csv -- python tools/conv_bench.py 10 64 ${BATCH:-1024} > $out/p$i.log 2>&1 || exit 1
done
