#!/bin/bash
# GPU step: PMC passes (kernel-trace only, one counter group per pass) of bk_conv3x3 at the
# self-play shape (256 boards, 64 -> 64 channels, relu epilogue), via tools/conv_bench.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_conv
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/pmc_conv/p$i -o c --output-format csv -- python tools/conv_bench.py 20 64 256 > gpurun_out/pmc_conv/p$i.log 2>&1 || exit 1
done
