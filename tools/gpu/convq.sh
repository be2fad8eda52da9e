#!/bin/bash
# Quick conv iteration: conv GPU tests, form-2 timing, form-2 phase stamps.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_conv.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_conv.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/conv_bench.py 200 64 ${BATCH:-256} > gpurun_out/conv_2.json 2>/dev/null
rc=$?; echo "form 2 rc=$rc $(cat gpurun_out/conv_2.json)"
[ $rc -ne 0 ] && exit $rc
BK_LIB=blokus_rl_amd/_lib/exp/libst.so timeout -k 10 120 python tools/wino_stamps.py ${BATCH:-256} > gpurun_out/stamps_2.json 2> gpurun_out/stamps_2.err
rc=$?; echo "stamps rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/stamps_2.json'))
print({k: (v['p50'], v['max']) if isinstance(v, dict) else v for k, v in d.items()})"
exit $rc
