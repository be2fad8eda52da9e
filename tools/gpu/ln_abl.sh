#!/bin/bash
# k_leafnet_x3 timing ablations (diagnostic builds, wrong outputs): per-launch us of the default and
# _lib/var/libln_abl{1,2}.so (1: no grid writes or barriers between tower convs; 2: 1 without the
# epilogue arithmetic), interleaved, 256 boards
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2 3; do
  for lib in "" blokus_rl_amd/_lib/var/libln_abl1.so blokus_rl_amd/_lib/var/libln_abl2.so; do
    echo "lib [$lib] $(BK_LIB=$lib timeout -k 10 120 python tools/leafnet_bench.py 50 256 2>/dev/null | cut -c1-200)"
  done
done
