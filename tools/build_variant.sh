#!/bin/bash
# A/B variant of the engine library: one source file recompiled with extra -D flags and linked with
# the other in-tree objects into blokus_rl_amd/_lib/exp/libln_<name>.so (tools/gpu/ln_variants.sh
# times every libln_*.so). Usage: tools/build_variant.sh <name> <source.hip> "<flags>" [<name> <src> "<flags>" ...]
set -e
cd "$(dirname "$0")/../blokus_rl_amd/csrc"
mkdir -p ../_lib/exp /tmp/bkvar
while [ $# -ge 3 ]; do
  name=$1; src=$2; flags=$3; shift 3
  base=$(basename $src .hip)
  OBJS=$(ls ../_lib/obj/*.o | grep -v "/$base.o")
  XF=""; [ "$base" = conv ] || [ "$base" = sims ] && XF="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function $XF $flags -c -o /tmp/bkvar/$name.o $src
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../_lib/exp/libln_$name.so $OBJS /tmp/bkvar/$name.o
done
rm -rf /tmp/bkvar
