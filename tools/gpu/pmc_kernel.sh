#!/bin/bash
# PMC passes of one kernel under one command, folded into a profiles-style JSON entry that
# bench.py reads (_pmc_traffic). One counter group per rocprofv3 run (FETCH_SIZE; WRITE_SIZE; two
# SQ groups), each under its own time limit; stops at the first failure.
#   tools/gpu/pmc_kernel.sh <out.json> <key> <kernel-name pattern> <units/launch> <algorithmic bytes/launch> \
#                           <note> <seconds per pass> -- <command...>
# e.g. tools/gpu/pmc_kernel.sh gpurun_out/r06_pmc.json k_vec_step7 k_vec_step7 8192 3219456 "..." 120 -- \
#      python bench.py --workload vecenv --vec-steps 100 --no-cpu-baseline
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
out=$1 key=$2 pat=$3 units=$4 algo=$5 note=$6 lim=$7
shift 7
[ "$1" = "--" ] && shift
dir=gpurun_out/pmc_$key
mkdir -p $dir
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL $lim rocprofv3 --pmc $grp --kernel-trace -d $dir/p$i -o c --output-format csv -- "$@" \
    > $dir/p$i.log 2>&1 || { echo "FAILED $key pass $i"; tail -5 $dir/p$i.log; exit 1; }
done
python tools/pmc_to_json.py "$out" "$key" "$pat" "$units" "$algo" "$note" $dir/p* || exit 1
rm -rf $dir/p?   # keep the logs only (per-dispatch CSVs can exceed gpurun's return size)
