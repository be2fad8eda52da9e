#!/bin/bash
# tools/leafnet_diff.py for the in-tree build and every variant library, at 20x20 and 14x14
cd "$GRAFT_REPO_ROOT" || exit 1
for lib in "" blokus_rl_amd/_lib/exp/libln_*.so; do
  n=${lib:+$(basename $lib .so)}; n=${n:-intree}
  for cfg in "256 20 5" "37 14 2"; do
    echo "== $n $cfg"
    BK_LIB=$lib timeout -k 10 120 python tools/leafnet_diff.py $cfg 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
