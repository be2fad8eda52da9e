#!/bin/bash
# HBM-side bytes of k_leaf_step_ov (the search kernel of the timed path) from rocprofv3 --pmc
# passes over the default self-play bench (FETCH_SIZE, WRITE_SIZE: separate passes), folded into
# gpurun_out/r04_pmc_leafstep.json (tools/pmc_to_json.py; bench.py reads it as search_roofline.traffic)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/pmc_step
mkdir -p $out
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $grp -d $out/p$i -o c --output-format csv -- python bench.py --workload selfplay --no-cpu-baseline --late-plies 0 > $out/p$i.log 2>&1 || { tail -5 $out/p$i.log; exit 1; }
  echo "pass $i ok"
done
python tools/pmc_to_json.py gpurun_out/r04_pmc_leafstep.json k_leaf_step_ov k_leaf_step_ov 256 0 "rocprofv3 --pmc passes of bench.py --workload selfplay (default plies): the mean over every k_leaf_step_ov dispatch of the run (graph replays and the eager timing launches); FETCH_SIZE doubled per the gfx950 16-B/lane correction (the W-row loads); other access widths uncalibrated" $out/p*
