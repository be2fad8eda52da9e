#!/bin/bash
# The learner's bk_conv_x3 path: its GPU tests, the learner A/B (base / cl+nativebn / x3), the
# train bench line, and a kernel-trace summary of the x3 learner step.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_train_conv_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tc_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -12 gpurun_out/tc_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/learner_ab.py --batch 1024 --steps 20 > gpurun_out/tc_ab.jsonl 2> gpurun_out/tc_ab.err
rc=$?; echo "ab rc=$rc"; cut -c1-200 gpurun_out/tc_ab.jsonl
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload train --no-cpu-baseline > gpurun_out/tc_train.json 2> gpurun_out/tc_train.err
rc=$?; echo "train rc=$rc"; cut -c1-900 gpurun_out/tc_train.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tc -o tc --output-format csv -- python tools/learner_ab.py --batch 1024 --steps 10 --configs x3 > gpurun_out/prof_tc.log 2>&1
rc=$?; echo "rocprof rc=$rc"; head -16 gpurun_out/prof_tc/tc_kernel_stats.csv | cut -c1-150
exit $rc
