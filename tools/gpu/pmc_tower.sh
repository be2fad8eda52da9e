#!/bin/bash
# GPU step: HBM-traffic PMC passes (kernel-trace only, one counter group per pass) of k_tower_wino
# at the self-play shape (256 boards, 5 blocks), via tools/tower_bench.py -> profiles/r01_pmc_tower.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/pmc_tower
mkdir -p $out
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $out/p$i -o c --output-format csv -- python tools/tower_bench.py 5 256 5 > $out/p$i.log 2>&1 || exit 1
done
python tools/pmc_to_json.py gpurun_out/r01_pmc_tower.json k_tower_wino k_tower_wino 256 55050240 \
  "rocprofv3 --pmc passes of tools/tower_bench.py (bk_resnet_tower, 256 boards 20x20, 10 convs 64->64); FETCH_SIZE doubled per the gfx950 correction, WRITE_SIZE as is; algorithmic bytes = tower input 26.2 MB + output 26.2 MB + 10 layers of Winograd U (262 KB each); the 9 intermediate activations (26.2 MB each way) stay on chip when L2 holds them" $out/p*
