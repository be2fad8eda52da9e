#!/bin/bash
# bench.py --workload train alone (the learner line).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload train --no-cpu-baseline > gpurun_out/train_only.json 2> gpurun_out/train_only.err
rc=$?; echo "train rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/train_only.json'));print(d['value'],d['roofline'],d.get('loss_roofline',{}).get('frac'))"
exit $rc
