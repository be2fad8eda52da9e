#!/bin/bash
# k_leafnet_x3p phase stamps (diagnostic library) and the launch time of the shipped one.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/lnp
BK_LN_PP=1 BK_LIB=blokus_rl_amd/_lib/exp/liblnst.so timeout -k 10 120 python tools/lnp_stamps.py 256 > gpurun_out/lnp/stamps.json 2> gpurun_out/lnp/stamps.err || { tail gpurun_out/lnp/stamps.err; exit 1; }
cat gpurun_out/lnp/stamps.json
for i in 1 2; do
  timeout -k 10 120 python tools/leafnet_bench.py 200 256 2>> gpurun_out/lnp/time.err | sed 's/^/w4 /' || exit 1
  BK_LN_PP=1 timeout -k 10 120 python tools/leafnet_bench.py 200 256 2>> gpurun_out/lnp/time.err | sed 's/^/pp /' || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_vecenv_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/lnp/vec_pytest.log 2>&1 || { tail -30 gpurun_out/lnp/vec_pytest.log; exit 1; }
tail -2 gpurun_out/lnp/vec_pytest.log
timeout -k 10 300 python bench.py --workload vecenv --no-cpu-baseline > gpurun_out/lnp/vec.json 2> gpurun_out/lnp/vec.err || { tail gpurun_out/lnp/vec.err; exit 1; }
cut -c1-400 gpurun_out/lnp/vec.json
BK_VEC_WAVE=1 timeout -k 10 300 python bench.py --workload vecenv --no-cpu-baseline > gpurun_out/lnp/vec_wave.json 2> gpurun_out/lnp/vec.err || { tail gpurun_out/lnp/vec.err; exit 1; }
cut -c1-300 gpurun_out/lnp/vec_wave.json
# VGPR accumulators in the 4-wave kernel (libvacc.so) vs the shipped AGPR form: bitwise + time
timeout -k 10 120 python tools/leafnet_ab.py dump gpurun_out/lnp/base.pt > gpurun_out/lnp/dump.log 2>&1 || exit 1
BK_LIB=blokus_rl_amd/_lib/exp/libvacc.so timeout -k 10 120 python tools/leafnet_ab.py dump gpurun_out/lnp/vacc.pt >> gpurun_out/lnp/dump.log 2>&1 || exit 1
python tools/leafnet_ab.py cmp gpurun_out/lnp/base.pt gpurun_out/lnp/vacc.pt
for i in 1 2; do
  timeout -k 10 120 python tools/leafnet_bench.py 200 256 2>> gpurun_out/lnp/time.err | sed 's/^/agpr /' || exit 1
  BK_LIB=blokus_rl_amd/_lib/exp/libvacc.so timeout -k 10 120 python tools/leafnet_bench.py 200 256 2>> gpurun_out/lnp/time.err | sed 's/^/vacc /' || exit 1
done
# per-tree phases of k_leaf_step_ov mid-game (diag build): median vs slowest tree
for p in 8 16; do
  BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so timeout -k 10 300 python tools/stamp_step_ov.py $p > gpurun_out/lnp/step_ov_$p.json 2>> gpurun_out/lnp/step.err || { tail gpurun_out/lnp/step.err; exit 1; }
  cut -c1-700 gpurun_out/lnp/step_ov_$p.json
done
