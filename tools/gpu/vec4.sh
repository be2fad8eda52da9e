#!/bin/bash
# k_vec_step7: bitwise tests vs the one-wave-per-env kernel, per-phase stamps, device step time (graph replay)
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/vec4
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_vecenv_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
grep -E "passed|failed" $out/pytest.log | tail -1
BK_LIB=blokus_rl_amd/_lib/exp/libvecst.so timeout -k 10 120 python tools/vec_stamps.py > $out/stamps.json 2> $out/stamps.err || { tail $out/stamps.err; exit 1; }
cat $out/stamps.json
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload vecenv --no-cpu-baseline > $out/bench_$i.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$out/bench_$i.json')); print('graph', round(d['value']/1e6,1), 'M/s', round(d['roofline']['kernel_ms']*1e3,2), 'us/step; eager', round(d['eager_env_step_calls']['value']/1e6,1))"
done
