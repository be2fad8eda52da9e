#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for w in 4 41 42; do
  export BK_LEGAL_WPB=$w
  timeout -k 10 200 python bench.py --workload legal --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/abl_$w.json 2> gpurun_out/abl_$w.err
  rc=$?; echo "wpb $w rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/abl_$w.json'));print(d['roofline']['kernel_ms'])"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
