#!/bin/bash
# Round-5 PMC refresh of the shipped kernels (one counter group per rocprofv3 run, each under its
# own time limit; stops at the first failure):
#   k_leafnet_x3 (tools/w3/run_w3.py x3: 256 boards, ResNet-5x64)   -> gpurun_out/r05_pmc_leafnet.json
#   k_legal_mask_rows<1,0,0> (bench.py --workload legal, 4096)      -> gpurun_out/r05_pmc_legal.json
#   k_leaf_step_ov (bench.py --workload selfplay, default window)  -> gpurun_out/r05_pmc_leafstep.json
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
set -o pipefail
run_passes() {  # <outdir> <limit> <cmd...>: FETCH_SIZE, WRITE_SIZE and two SQ groups
  local out=$1 lim=$2; shift 2
  mkdir -p $out
  local i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL $lim rocprofv3 --pmc $grp --kernel-trace -d $out/p$i -o c --output-format csv -- "$@" > $out/p$i.log 2>&1 || { echo "FAILED $out pass $i"; tail -5 $out/p$i.log; return 1; }
  done
  echo "$out ok"
}
run_passes gpurun_out/pmc5_leafnet 120 python tools/w3/run_w3.py 5 x3 || exit 1
python tools/pmc_to_json.py gpurun_out/r05_pmc_leafnet.json k_leafnet_x3 k_leafnet_x3 256 5677056 "round 5: rocprofv3 --pmc passes of tools/w3/run_w3.py 5 x3 (256 boards, ResNet-5x64, the shipped build with the x0 stash in LDS); algorithmic bytes = observations 3,276,800 + split weights 1,506,304 (stem 24,576 + 10 convs x 147,456 + heads 102,400 + biases/scales) + pf/v out 823,296" gpurun_out/pmc5_leafnet/p* || exit 1
BK_LEGAL_WPB=1 run_passes gpurun_out/pmc5_legal 240 python bench.py --workload legal --steps 20 --warmup 2 --no-cpu-baseline --graph 0 || exit 1
python tools/pmc_to_json.py gpurun_out/r05_pmc_legal.json k_legal_mask k_legal_mask 4096 17186816 "round 5: rocprofv3 --pmc passes of bench.py --workload legal (eager launches, 4096 boards) on the shipped k_legal_mask_rows<1,0,0>; algorithmic bytes = 4096 x (384 state + 3808 mask + 4 count)" gpurun_out/pmc5_legal/p* || exit 1
run_passes gpurun_out/pmc5_step 400 python bench.py --workload selfplay --no-cpu-baseline --late-plies 0 || exit 1
python tools/pmc_to_json.py gpurun_out/r05_pmc_leafstep.json k_leaf_step_ov k_leaf_step_ov 256 0 "round 5: rocprofv3 --pmc passes of bench.py --workload selfplay (default window, plies 5-30): the mean over every k_leaf_step_ov dispatch of the run; FETCH_SIZE doubled per the gfx950 16-B/lane correction (the W-row loads); algorithmic_bytes: the addressed bytes per launch of the bench's search_roofline (filled from its output)" gpurun_out/pmc5_step/p* || exit 1
# keep the summaries only (the per-dispatch CSVs of a self-play run exceed gpurun's 64-MiB return)
rm -rf gpurun_out/pmc5_leafnet/p? gpurun_out/pmc5_legal/p? gpurun_out/pmc5_step/p?
echo done
