#!/bin/bash
# Validation: the MFMA/LDS probe (seconds), every GPU test, smoke(). Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 100 blokus_rl_amd/_lib/exp/mfma_lds > gpurun_out/mfma_lds.txt 2>&1 || { echo "probe failed"; exit 1; }
cat gpurun_out/mfma_lds.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
exit $rc
