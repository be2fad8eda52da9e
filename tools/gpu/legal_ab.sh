#!/bin/bash
# k_legal_mask_rows: bit-exactness of the lean variant (BK_LEGAL_WPB=41) and of the diagnostic
# store-order build, then per-launch times (tools/legal_scale.py) of the default, the lean variants
# (41-44) and the timing ablations (_lib/var/liblegal_abl<k>.so: 1 no orientation work, 2 no mask
# stores, 4 LDS reads of a board before its stores)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/legal_ab.txt
: > $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_env_gpu.py \
  -k "benchmark_boards or variants_bit_exact" >> $out 2>&1 || { echo "tests failed"; tail -20 $out; exit 1; }
BK_LIB=blokus_rl_amd/_lib/var/liblegal_abl4.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread tests/test_env_gpu.py -k "benchmark_boards" >> $out 2>&1 || { echo "abl4 tests failed"; tail -20 $out; exit 1; }
run() {  # label, env...
  local label=$1; shift
  echo -n "$label " >> $out
  env "$@" timeout -k 10 120 python tools/legal_scale.py 1024 4096 16384 >> $out 2>&1 || { echo "$label failed"; return 1; }
}
for rep in 1 2; do
  run default BK_LEGAL_WPB=1 && run lean41 BK_LEGAL_WPB=41 && run lean42 BK_LEGAL_WPB=42 \
    && run lean43 BK_LEGAL_WPB=43 && run nt44 BK_LEGAL_WPB=44 \
    && run abl1 BK_LIB=blokus_rl_amd/_lib/var/liblegal_abl1.so \
    && run abl2 BK_LIB=blokus_rl_amd/_lib/var/liblegal_abl2.so \
    && run abl4 BK_LIB=blokus_rl_amd/_lib/var/liblegal_abl4.so \
    && run abl4lean42 BK_LIB=blokus_rl_amd/_lib/var/liblegal_abl4.so BK_LEGAL_WPB=42 \
    && run abl1lean42 BK_LIB=blokus_rl_amd/_lib/var/liblegal_abl1.so BK_LEGAL_WPB=42 || exit 1
done
grep -E "passed|failed|us_per_launch" $out
