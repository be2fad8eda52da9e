#!/bin/bash
# GPU step: kernel-level profile of the leaf evaluator (LeafResNet graph replays).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/nnprof -o nn --output-format csv -- python tools/nn_profile.py 200 > gpurun_out/nnprof.log 2>&1
