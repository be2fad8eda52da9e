#!/bin/bash
# k_leafnet_x3 at the self-play shape: event timing, per-wave phase stamps (diagnostic build), PMC passes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/pmc_leafnet
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_leafnet_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 120 python tools/leafnet_bench.py 200 256 > $out/time.json 2> $out/time.err || exit 1
cat $out/time.json
BK_LIB=blokus_rl_amd/_lib/exp/liblnst.so timeout -k 10 120 python tools/leafnet_bench.py 50 256 --stamps > $out/stamps.json 2> $out/stamps.err || exit 1
cat $out/stamps.json
[ -n "$NO_PMC" ] && exit 0
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $out/p$i -o c --output-format csv -- python tools/leafnet_bench.py 5 256 > $out/p$i.log 2>&1 || exit 1
done
python tools/pmc_to_json.py gpurun_out/r04_pmc_leafnet.json k_leafnet_x3 k_leafnet_x3 256 0 "rocprofv3 --pmc passes of tools/leafnet_bench.py" $out/p*
