#!/bin/bash
# descent / expansion phase cycles (BK_STAMPS build) after 4 and 15 plies of the bench config
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/stamp_search
for p in 4 15; do
  BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so timeout -k 10 300 python tools/stamp_search.py $p > gpurun_out/stamp_search/ply$p.txt 2>&1 || { tail gpurun_out/stamp_search/ply$p.txt; exit 1; }
  echo "== ply $p"; cat gpurun_out/stamp_search/ply$p.txt
done
