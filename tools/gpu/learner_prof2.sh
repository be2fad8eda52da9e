#!/bin/bash
# Kernel breakdown of the learner step at batch 1024 with channels_last + native batch norm.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_learner2 -o l2 --output-format csv -- python tools/learner_ab.py --batch 1024 --steps 10 --configs ${LAB_CFG:-cl+nativebn} > gpurun_out/prof_learner2.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep config gpurun_out/prof_learner2.log
exit $rc
