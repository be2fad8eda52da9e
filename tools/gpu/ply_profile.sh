#!/bin/bash
# kernel trace of the driver's self-play arguments (20 timed plies after 5): per-ply net / leaf
# step / tail time (tools/ply_profile.py)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_ply -o ply --output-format csv -- python bench.py --workload selfplay --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_ply.log 2>&1 || { tail -5 gpurun_out/prof_ply.log; exit 1; }
python tools/ply_profile.py gpurun_out/prof_ply/ply_kernel_trace.csv
