#!/bin/bash
# k_leafnet_w3 / x3 iteration: leaf-net parity tests, x3/w3 timing A/B, w3 stamps. Later steps only
# after a normal pytest exit (0 passed / 1 failed).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_leafnet_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_w3.log 2>&1
rc=$?; echo "leafnet pytest rc=$rc"; tail -4 gpurun_out/pytest_w3.log | cut -c1-300
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python tools/w3/bench_w3.py 100 3 > gpurun_out/bench_w3.json 2> gpurun_out/bench_w3.err
rc2=$?; echo "bench_w3 rc=$rc2"; cat gpurun_out/bench_w3.json
[ $rc2 -ne 0 ] && exit $rc2
BK_LIB=blokus_rl_amd/_lib/exp/libw3st.so timeout -k 10 200 python tools/w3/stamps_w3.py > gpurun_out/w3_stamps.json 2> gpurun_out/w3_stamps.err
rc3=$?; echo "stamps rc=$rc3"
python -c "import json; d=json.load(open('gpurun_out/w3_stamps.json')); [print(k, d[k]) for k in d if k.startswith('unit')]; print('l1_total', d['l1_total'], 'total', d['total'])"
exit $rc
