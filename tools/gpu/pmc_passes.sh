#!/bin/bash
# Four rocprofv3 --pmc passes of one command (FETCH_SIZE; WRITE_SIZE; two SQ groups), one counter
# group per run, each under its own time limit, into <dir>/p1..p4 (fold them with
# tools/pmc_to_json.py, one call per kernel). Stops at the first failure.
#   tools/gpu/pmc_passes.sh <dir> <seconds per pass> -- <command...>
export TMPDIR=/tmp
dir=$1 lim=$2
shift 2
[ "$1" = "--" ] && shift
mkdir -p $dir
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "pmc pass $i: $*"
  timeout -s KILL $lim rocprofv3 --pmc $grp --kernel-trace -d $dir/p$i -o c --output-format csv -- "$@" \
    > $dir/p$i.log 2>&1 || { echo "FAILED pass $i"; tail -5 $dir/p$i.log; exit 1; }
done
