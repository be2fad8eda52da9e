#!/bin/bash
# Time every k_leafnet_x3 variant library under blokus_rl_amd/_lib/exp/libln_*.so (and the
# in-tree build), 200 launches each at the self-play shape; A/B-dump each against the in-tree build.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/lnvar
mkdir -p $out
export TMPDIR=/tmp
# reference outputs: a saved dump of an earlier build (blokus_rl_amd/_lib/exp/ref.pt), else the in-tree build
timeout -k 10 120 python tools/leafnet_ab.py dump $out/intree.pt > $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
if [ -f blokus_rl_amd/_lib/exp/ref.pt ]; then cp blokus_rl_amd/_lib/exp/ref.pt $out/ref.pt; else cp $out/intree.pt $out/ref.pt; fi
python tools/leafnet_ab.py cmp $out/ref.pt $out/intree.pt > $out/intree.cmp 2>&1; echo "intree cmp=$?"
echo "intree $(timeout -k 10 120 python tools/leafnet_bench.py 200 256 2>>$out/err)" || exit 1
for lib in blokus_rl_amd/_lib/exp/libln_*.so; do
  n=$(basename $lib .so)
  BK_LIB=$lib timeout -k 10 120 python tools/leafnet_ab.py dump $out/$n.pt >> $out/dump.log 2>&1 || { echo "$n dump failed"; tail $out/dump.log; exit 1; }
  python tools/leafnet_ab.py cmp $out/ref.pt $out/$n.pt > $out/$n.cmp 2>&1; c=$?
  echo "$n cmp=$c $(BK_LIB=$lib timeout -k 10 120 python tools/leafnet_bench.py 200 256 2>>$out/err)" || exit 1
done
if [ -f blokus_rl_amd/_lib/exp/libln_st.so ]; then
  BK_LIB=blokus_rl_amd/_lib/exp/libln_st.so timeout -k 10 120 python tools/leafnet_bench.py 50 256 --stamps 2>>$out/err || exit 1
fi
