#!/bin/bash
# GPU step: FETCH_SIZE / WRITE_SIZE passes (kernel-trace only) of bk_conv3x3 at the self-play
# shape (256 boards, 64 -> 64, even N -> the Winograd form) -> gpurun_out/pmc_wino_t/p*.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/pmc_wino_t
mkdir -p $out
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --kernel-trace -d $out/p$i -o c --output-format csv -- python tools/conv_bench.py 20 64 256 > $out/p$i.log 2>&1 || exit 1
done
