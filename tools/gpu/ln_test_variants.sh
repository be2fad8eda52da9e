#!/bin/bash
# k_leafnet_x3 accuracy test (tests/test_leafnet_gpu.py) for the in-tree build and every variant
# library under blokus_rl_amd/_lib/exp/libln_*.so
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/lntest; mkdir -p $out
for lib in "" blokus_rl_amd/_lib/exp/libln_*.so; do
  n=${lib:+$(basename $lib .so)}; n=${n:-intree}
  BK_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_leafnet_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/$n.log 2>&1
  echo "$n rc=$? $(tail -1 $out/$n.log)"
done
