#!/bin/bash
# k_vec_step7 phase stamps (16 and 8 lanes) and the 4-wave leaf net's stamps / clock
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/diag3
mkdir -p $out
for g in 16 8; do
  BK_VEC_LANES=$g BK_LIB=blokus_rl_amd/_lib/exp/libvecst.so timeout -k 10 120 python tools/vec_stamps.py > $out/vec_$g.json 2> $out/vec.err || { tail $out/vec.err; exit 1; }
  echo "lanes $g"; cat $out/vec_$g.json
done
BK_LIB=blokus_rl_amd/_lib/exp/liblnst.so timeout -k 10 120 python tools/leafnet_bench.py 50 256 --stamps > $out/ln.json 2> $out/ln.err || { tail $out/ln.err; exit 1; }
cut -c1-1500 $out/ln.json
timeout -k 10 300 python bench.py --workload vecenv --no-cpu-baseline > $out/vec_bench.json 2> $out/vec_bench.err || { tail $out/vec_bench.err; exit 1; }
python -c "import json; d=json.load(open('$out/vec_bench.json')); print('graph', round(d['value']/1e6,1), 'M/s', round(d['roofline']['kernel_ms']*1e3,2), 'us/step; eager', round(d['eager_env_step_calls']['value']/1e6,1))"
