#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_env_gpu.py tests/test_mcts_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_legal.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_legal.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for impl in w1 w2 w4 w8 items; do
  if [ $impl = items ]; then export BK_LEGAL_KERNEL=items; else unset BK_LEGAL_KERNEL; export BK_LEGAL_WPB=${impl#w}; fi
  timeout -k 10 200 python bench.py --workload legal --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/bench_legal_$impl.json 2> gpurun_out/bench_legal_$impl.err
  rc=$?; echo "bench $impl rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/bench_legal_$impl.json'));print(d['value'], d['roofline'])"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
unset BK_LEGAL_KERNEL BK_LEGAL_WPB
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_legal2 -o legal --output-format csv -- python bench.py --workload legal --steps 200 --warmup 20 --no-cpu-baseline --graph 0 > gpurun_out/prof_legal2.log 2>&1
rc=$?; echo "rocprof rc=$rc"; head -4 gpurun_out/prof_legal2/legal_kernel_stats.csv | cut -c1-160
exit $rc
