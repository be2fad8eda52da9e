#!/bin/bash
# GPU step: kernel-level profile of the self-play workload alone.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/spprof -o sp --output-format csv -- python bench.py --workload selfplay --no-cpu-baseline --steps 5 > gpurun_out/spprof.log 2>&1
