#!/bin/bash
# The bench as the driver runs it (N=1), optionally followed by the same command under
# rocprofv3 --kernel-trace --stats (PROFILE=1; the stats CSV -> gpurun_out/bench_kernel_stats.csv).
#   tools/gpu/bench.sh [steps] [warmup]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${1:-20} W=${2:-5}
timeout -k 10 420 python bench.py --gpus 1 --steps $S --warmup $W > gpurun_out/bench.json 2> gpurun_out/bench.err \
  || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ "${PROFILE:-0}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/bench_kt -o kt --output-format csv -- python bench.py --gpus 1 --steps $S --warmup $W \
    > gpurun_out/bench_kt.json 2> gpurun_out/bench_kt.err || { tail -20 gpurun_out/bench_kt.err; exit 1; }
  for f in $(find /tmp/bench_kt -name "*kernel_stats.csv"); do grep -q k_leaf_step_ov $f && cp $f gpurun_out/bench_kernel_stats.csv; done
  head -12 gpurun_out/bench_kernel_stats.csv | cut -c1-160
fi
