#!/bin/bash
# per-tree phase cycles of k_leaf_step_ov (BK_STAMPS build) after 6 / 15 / 25 plies of the bench config
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/stamp_ov
mkdir -p $out
for p in 6 15 25; do
  BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so timeout -k 10 200 python tools/stamp_step_ov.py $p > $out/ply$p.json 2> $out/ply$p.err || { tail $out/ply$p.err; exit 1; }
  echo "ply $p"; cut -c1-4000 $out/ply$p.json
done
