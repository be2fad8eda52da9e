#!/bin/bash
# the fused ply tail (ply.hip): self-play GPU tests, then the self-play bench with and without it
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ply
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_selfplay_gpu.py > gpurun_out/ply/pytest.log 2>&1
rc=$?; tail -12 gpurun_out/ply/pytest.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0 1 0; do
  BK_PLY_FUSED=$f timeout -k 10 200 python bench.py --workload selfplay --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/ply/b$f.json 2> gpurun_out/ply/b$f.err || { tail -5 gpurun_out/ply/b$f.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ply/b$f.json')); print('fused=$f', round(d['value']), round(d['ms_per_step'],3))"
done
