#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
BK_LIB=blokus_rl_amd/_lib/exp/libw3st.so timeout -k 10 200 python tools/w3/stamps_w3.py > gpurun_out/w3_stamps.json 2> gpurun_out/w3_stamps.err
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/w3_stamps.json; tail -3 gpurun_out/w3_stamps.err
exit $rc
