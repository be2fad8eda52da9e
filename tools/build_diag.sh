#!/bin/bash
# The BK_STAMPS build of the engine (per-tree phase stamps, tools/stamp_step_ov.py) into
# blokus_rl_amd/_lib/diag/libblokus_hip_diag.so; the objects in parallel. Run from the repo root
# after `make` (tables.o comes from the regular build).
set -e
cd blokus_rl_amd/csrc
mkdir -p ../_lib/diag/o
rm -f ../_lib/diag/o/*.o
pids=()
for f in env.hip mcts.hip vecenv.hip train.hip trainconv.hip trainbn.hip trainfc.hip ppo.hip netops.hip conv.hip leafnet.hip leafnet_w3.hip ply.hip; do
  XF=""; [ "$f" = conv.hip ] && XF="-fno-slp-vectorize"; [ "$f" = leafnet_w3.hip ] && XF="-mllvm -pragma-unroll-threshold=1000000"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function -DBK_STAMPS $XF \
    -c -o ../_lib/diag/o/$f.o $f &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
cp ../_lib/obj/tables.o ../_lib/diag/o/
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../_lib/diag/libblokus_hip_diag.so ../_lib/diag/o/*.o
