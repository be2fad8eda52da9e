#!/bin/bash
# k_leafnet_x3 A/B: the in-tree build against blokus_rl_amd/_lib/exp/libln_<name>.so for each name
# given (bitwise outputs, then per-launch time interleaved twice), then the leaf-net GPU tests.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/epi; mkdir -p $out
timeout -k 10 120 python tools/leafnet_ab.py dump $out/tree.pt > $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
for n in "$@"; do
  BK_LIB=blokus_rl_amd/_lib/exp/libln_$n.so timeout -k 10 120 python tools/leafnet_ab.py dump $out/$n.pt >> $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
  echo "== tree vs $n"; python tools/leafnet_ab.py cmp $out/tree.pt $out/$n.pt
done
for rep in 1 2; do
  echo "tree $(timeout -k 10 120 python tools/leafnet_bench.py 300 256)" || exit 1
  for n in "$@"; do
    echo "$n $(BK_LIB=blokus_rl_amd/_lib/exp/libln_$n.so timeout -k 10 120 python tools/leafnet_bench.py 300 256)" || exit 1
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_leafnet_gpu.py > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; exit $rc
