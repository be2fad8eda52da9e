cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for mode in "0 0" "1 1" "1 10" "1 0"; do
  set -- $mode
  BK_SIM_FUSED=$1 BK_SIMS_PER_LAUNCH=$2 timeout -k 10 240 python bench.py --workload selfplay --no-cpu-baseline > gpurun_out/bench_mode_$1_$2.json 2>gpurun_out/bench_mode_$1_$2.err || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/bench_mode_$1_$2.json')); r=d['roofline']; print('fused=$1 per_launch=$2', round(d['value']), r.get('kernel','')[:20], round(r.get('kernel_ms',0),3), round(r.get('frac',0),3))"
done
