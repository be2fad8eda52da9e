#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_mcts_gpu.py tests/test_env_gpu.py tests/test_selfplay_gpu.py tests/test_dropin_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_search.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_search.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --workload selfplay --model dumbnet --no-cpu-baseline > gpurun_out/b_dumb.json 2> gpurun_out/b_dumb.err
rc=$?; echo "dumb rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/b_dumb.json'));print(d['value'], d['stage_ms_per_sim_step'], d['roofline']['frac'])"
exit $rc
