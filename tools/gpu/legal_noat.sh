cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/legalvar
for lib in "" blokus_rl_amd/_lib/exp/libnoat.so; do
  BK_LIB=$lib timeout -k 10 120 python bench.py --workload legal --no-cpu-baseline > gpurun_out/legalvar/x.json 2> gpurun_out/legalvar/x.err || { tail -3 gpurun_out/legalvar/x.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/legalvar/x.json')); r=d['roofline']; print('lib [$lib]', round(r['kernel_ms']*1e3,2), 'us')"
done
