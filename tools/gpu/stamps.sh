#!/bin/bash
# Winograd conv phase stamps (diagnostics build) for form 2 and form 1, then the stall-counter passes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for f in 2 1; do
  BK_CONV_WINO=$f BK_LIB=blokus_rl_amd/_lib/exp/libst.so timeout -k 10 120 python tools/wino_stamps.py ${BATCH:-256} > gpurun_out/stamps_$f.json 2> gpurun_out/stamps_$f.err
  rc=$?; echo "stamps form $f rc=$rc"; cat gpurun_out/stamps_$f.json
  [ $rc -ne 0 ] && exit $rc
done
[ -n "$NO_PMC" ] && exit 0
BATCH=${BATCH:-256} tools/gpu/pmc_wino.sh
rc=$?; echo "pmc rc=$rc"
python tools/pmc_summary.py gpurun_out/pmc_wino wino2 2>&1 | tail -30
exit $rc
