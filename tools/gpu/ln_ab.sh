#!/bin/bash
# k_leafnet_x3: tests, then this build vs BK_LIB=$1 interleaved (tools/leafnet_bench.py, 256 boards)
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/ln_ab
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_leafnet_gpu.py tests/test_dropin_gpu.py -k "leafnet or predict or x3" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for i in 1 2 3; do
  for lib in "" "$1"; do
    BK_LIB=$lib timeout -k 10 120 python tools/leafnet_bench.py 300 256 > $out/l.json 2> $out/l.err || { tail -3 $out/l.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$out/l.json')); print('lib [%s]' % sys.argv[1], round(d['us_per_launch'],2), 'us', round(d['frac_of_2.5PF'],3))" "$lib"
  done
done
