#!/bin/bash
# Kernel-trace of a short self-play bench; the launch gaps between the sim-step's kernels
# (leaf net -> leaf step -> next leaf net) and the per-ply time outside them (tools/trace_gaps.py).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_gaps -o gaps --output-format csv -- python bench.py --workload selfplay --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/prof_gaps.log 2>&1 || { tail -5 gpurun_out/prof_gaps.log; exit 1; }
python tools/trace_gaps.py gpurun_out/prof_gaps/gaps_kernel_trace.csv
