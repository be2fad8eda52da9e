#!/bin/bash
# SQ counter passes of k_leafnet_x3g and k_leafnet_x3 (tools/x3g_bench.py, 10 reps each)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmcx3g
export TMPDIR=/tmp
CMD="python tools/x3g_bench.py 256 10"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmcx3g/p$i -o p -- $CMD > gpurun_out/pmcx3g/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmcx3g/p$i.log; exit $rc; fi
done
python tools/pmc_summary.py gpurun_out/pmcx3g k_leafnet_x3gILi
python tools/pmc_summary.py gpurun_out/pmcx3g k_leafnet_x3ILi
