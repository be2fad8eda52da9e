#!/bin/bash
# config-2 legal kernel: tests, then this build vs BK_LIB=$1 interleaved (bench --workload legal)
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/legal_ab
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for i in 1 2 3; do
  for lib in "" "$1"; do
    BK_LIB=$lib timeout -k 10 120 python bench.py --workload legal --no-cpu-baseline > $out/l.json 2> $out/l.err || { tail -3 $out/l.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$out/l.json')); r=d['roofline']; print('lib [%s]' % sys.argv[1], round(d['value']/1e6,1), 'M boards/s', round(r['kernel_ms']*1e3,2), 'us frac', round(r['frac'],3))" "$lib"
  done
done
