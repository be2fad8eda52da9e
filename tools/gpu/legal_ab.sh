#!/bin/bash
# k_legal_mask_rows: bit-exactness of every variant, then per-launch times (tools/legal_scale.py) of
# the default (the lean step), round 4's step (40) and the lean step on 3 / 2 waves per group (45 / 46)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/legal_ab.txt
: > $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_env_gpu.py \
  -k "benchmark_boards or variants_bit_exact" >> $out 2>&1 || { echo "tests failed"; tail -20 $out; exit 1; }
run() {  # label, env...
  local label=$1; shift
  echo "$label $(env "$@" timeout -k 10 120 python tools/legal_scale.py 1024 4096 16384 2>/dev/null)" >> $out
}
for rep in 1 2; do
  run default BK_LEGAL_WPB=1 && run r4step BK_LEGAL_WPB=40 \
    && run abl1_no_orient BK_LIB=blokus_rl_amd/_lib/var/liblegal_abl1.so \
    && run abl2_no_stores BK_LIB=blokus_rl_amd/_lib/var/liblegal_abl2.so \
    && run abl8_empty BK_LIB=blokus_rl_amd/_lib/var/liblegal_abl8.so || exit 1
done
grep -E "passed|failed|us_per_launch" $out
