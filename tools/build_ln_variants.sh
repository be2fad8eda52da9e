#!/bin/bash
# Build k_leafnet_x3 A/B variants: leafnet.hip compiled with the given -D flags, linked with the
# in-tree objects into blokus_rl_amd/_lib/exp/libln_<name>.so.  Usage: tools/build_ln_variants.sh name "-DX=1 ..." ...
set -e
cd "$(dirname "$0")/../blokus_rl_amd/csrc"
mkdir -p ../_lib/exp /tmp/lnvar
OBJS=$(ls ../_lib/obj/*.o | grep -v leafnet.o)
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function $flags -c -o /tmp/lnvar/$name.o leafnet.hip &
done
wait
for o in /tmp/lnvar/*.o; do
  n=$(basename $o .o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../_lib/exp/libln_$n.so $OBJS $o
done
rm -rf /tmp/lnvar
ls ../_lib/exp
