#!/bin/bash
# SQ counter passes of the config-2 legal kernel for each BK_LEGAL_WPB variant in $VARIANTS
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmcab
export TMPDIR=/tmp
CMD="python bench.py --workload legal --steps 20 --warmup 2 --no-cpu-baseline --graph 0"
for v in ${VARIANTS:-1 31}; do
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    BK_LEGAL_WPB=$v timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmcab/v${v}_p$i -o p -- $CMD > gpurun_out/pmcab/v${v}_p$i.log 2>&1
    rc=$?; echo "variant $v pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmcab/v${v}_p$i.log; exit $rc; fi
  done
done
