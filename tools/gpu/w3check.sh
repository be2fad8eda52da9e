#!/bin/bash
# quick k_leafnet_w3 correctness/timing check of the default library and the variants given
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/w3/check_w3.py > gpurun_out/w3check.txt 2>&1 || { echo "default failed"; tail -5 gpurun_out/w3check.txt; exit 1; }
for v in "$@"; do
  BK_LIB=blokus_rl_amd/_lib/var/$v.so timeout -k 10 120 python tools/w3/check_w3.py >> gpurun_out/w3check.txt 2>&1 || { echo "$v failed"; break; }
done
grep '^{' gpurun_out/w3check.txt
