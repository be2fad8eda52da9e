#!/bin/bash
# A/B builds: the engine with extra compile flags into blokus_rl_amd/_lib/exp/lib<NAME>.so (objects
# under /tmp), for tools/gpu/lib_ab.sh. Usage: tools/build_lib_variant.sh NAME "-DKNOB=1 ..." [SRC_DIR]
# (SRC_DIR: another checkout's csrc, e.g. a git worktree of the previous commit). Run from the repo root.
set -e
name=$1; flags=$2; src=${3:-blokus_rl_amd/csrc}
root=$(pwd)
obj=/tmp/bk_variant/$name
mkdir -p "$obj" blokus_rl_amd/_lib/exp
rm -f "$obj"/*.o
cd "$src"
pids=()
for f in env.hip mcts.hip vecenv.hip train.hip ppo.hip netops.hip conv.hip leafnet.hip ply.hip; do
  [ -f "$f" ] || continue
  XF=""; [ "$f" = conv.hip ] && XF="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function $XF $flags \
    -c -o "$obj/$f.o" $f &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
cp "$root/blokus_rl_amd/_lib/obj/tables.o" "$obj/"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$root/blokus_rl_amd/_lib/exp/lib$name.so" "$obj"/*.o
echo "built blokus_rl_amd/_lib/exp/lib$name.so"
