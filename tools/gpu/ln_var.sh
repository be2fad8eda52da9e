#!/bin/bash
# k_leafnet_x3 build variants: each library given must be bitwise equal to the default build
# (tools/leafnet_ab.py dump/cmp), then per-launch us of the default and the variants, interleaved
# (3 rounds, tools/leafnet_bench.py, 256 boards). Usage: tools/gpu/ln_var.sh <lib.so>...
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/lnvar
mkdir -p $out
timeout -k 10 120 python tools/leafnet_ab.py dump $out/base.pt > $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
for lib in "$@"; do
  BK_LIB=$lib timeout -k 10 120 python tools/leafnet_ab.py dump $out/v.pt >> $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
  echo "$lib: $(python tools/leafnet_ab.py cmp $out/base.pt $out/v.pt 2>&1 | tail -1)"
done
for r in 1 2 3; do
  for lib in "" "$@"; do
    echo "lib [$lib] $(BK_LIB=$lib timeout -k 10 120 python tools/leafnet_bench.py 50 256 2>/dev/null | cut -c1-120)"
  done
done
