#!/bin/bash
# config-2 legal-move kernel: every k_legal_mask_rows variant (BK_LEGAL_WPB) timed by bench.py
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/legalvar
for v in ${BK_LEGAL_VARIANTS:-11 1 2 4 8 21}; do
  BK_LEGAL_WPB=$v timeout -k 10 120 python bench.py --workload legal --no-cpu-baseline > gpurun_out/legalvar/$v.json 2> gpurun_out/legalvar/$v.err || { echo "$v failed"; tail -3 gpurun_out/legalvar/$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/legalvar/$v.json')); r=d['roofline']; print('wpb $v', round(d['value']/1e6,1), 'M boards/s', round(r['kernel_ms']*1e3,2), 'us', 'frac', round(r['frac'],3))"
done
