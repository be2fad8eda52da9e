#!/bin/bash
# The fused simulation path: its parity tests and one self-play bench line with BK_SIM_FUSED=1.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sims_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_fused.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_fused.log
[ $rc -ne 0 ] && exit $rc
BK_SIM_FUSED=1 timeout -k 10 240 python bench.py --workload selfplay --no-cpu-baseline > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err
rc=$?; python -c "
import json; d=json.load(open('gpurun_out/bench_fused.json')); r=d['roofline']; print(round(d['value']), round(r.get('kernel_ms',0),2), round(r.get('frac',0),3))"
exit $rc
