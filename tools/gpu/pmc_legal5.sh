#!/bin/bash
# PMC passes of the shipped config-2 legal kernel (round 5's lean step, k_legal_mask_rows<1,3,0,20>)
# -> gpurun_out/r05_pmc_legal_lean.json (one counter group per rocprofv3 run, own time limit each)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/pmc5_legal_lean
mkdir -p $out
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d $out/p$i -o c --output-format csv -- python bench.py --workload legal --steps 20 --warmup 2 --no-cpu-baseline --graph 0 > $out/p$i.log 2>&1 || { echo "FAILED pass $i"; tail -5 $out/p$i.log; exit 1; }
done
python tools/pmc_to_json.py gpurun_out/r05_pmc_legal_lean.json k_legal_mask "k_legal_mask_rows<1, 3, 0, 20>" 4096 17186816 "round 5: rocprofv3 --pmc passes of bench.py --workload legal (eager launches, 4096 boards) on the shipped lean step k_legal_mask_rows<1,3,0,20>; algorithmic bytes = 4096 x (384 state + 3808 mask + 4 count)" $out/p* || exit 1
rm -rf $out/p?
echo done
