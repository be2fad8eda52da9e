#!/bin/bash
# PMC passes of k_leafnet_w3 (one counter group per run) -> gpurun_out/w3_pmc.json
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/pmc_w3
mkdir -p $out
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $out/p$i -o c --output-format csv -- python tools/w3/run_w3.py 5 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
python tools/pmc_to_json.py gpurun_out/w3_pmc.json k_leafnet_w3 k_leafnet_w3 256 0 "rocprofv3 --pmc passes of tools/w3/run_w3.py" $out/p*
python -c "import json; d=json.load(open('gpurun_out/w3_pmc.json'))['kernels']['k_leafnet_w3']['counters_per_dispatch']; print(json.dumps({k: round(v) for k, v in d.items()}))"
