#!/bin/bash
# bitwise A/B of every variant library blokus_rl_amd/_lib/exp/libln_*.so against libbase.so
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/ab; mkdir -p $out
BK_LIB=blokus_rl_amd/_lib/exp/libbase.so timeout -k 10 120 python tools/leafnet_ab.py dump $out/base.pt > $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
for lib in blokus_rl_amd/_lib/exp/libln_*.so; do
  n=$(basename $lib .so)
  BK_LIB=$lib timeout -k 10 120 python tools/leafnet_ab.py dump $out/$n.pt >> $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
  echo "== $n"; python tools/leafnet_ab.py cmp $out/base.pt $out/$n.pt
done
exit 0
