#!/bin/bash
# Conv kernels: GPU tests, then per-form timing at the leaf batch (tools/conv_bench.py), then the
# self-play bench line. Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_conv.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_conv.log
[ $rc -ne 0 ] && exit $rc
for form in 2 1 d; do
  if [ $form = d ]; then env="BK_CONV_DIRECT=1"; elif [ $form = 1 ]; then env="BK_CONV_WINO=1"; else env="BK_CONV_WINO=2"; fi
  env $env timeout -k 10 120 python tools/conv_bench.py 200 64 ${BATCH:-256} > gpurun_out/conv_$form.json 2>/dev/null
  rc=$?; echo "form $form rc=$rc $(cat gpurun_out/conv_$form.json)"
  [ $rc -ne 0 ] && exit $rc
done
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python bench.py --workload selfplay --no-cpu-baseline > gpurun_out/bench_sp.json 2> gpurun_out/bench_sp.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/bench_sp.json
exit $rc
