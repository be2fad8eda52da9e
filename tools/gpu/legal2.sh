#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_env_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_legal.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_legal.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in 1 21 1 21; do
  export BK_LEGAL_WPB=$w
  timeout -k 10 200 python bench.py --workload legal --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/bl_$w.json 2> gpurun_out/bl_$w.err
  rc=$?; echo "wpb $w rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/bl_$w.json'));print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
