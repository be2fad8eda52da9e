#!/bin/bash
# Round 6 measurement set of the shipped build (every roofline number of the bench line from a
# committed profile): the bench as the driver runs it; the same command under --kernel-trace
# (stats + the timed window's per-kernel averages, tools/window_avg.py); PMC passes of the
# self-play kernels (k_leaf_step_ov over the window's launches, k_leafnet_x3), the config-2 legal
# kernel and the learner's kernels (k_conv_x3, k_conv_x3_wgrad, k_bn_*, k_policy_loss pair).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
( while true; do sleep 45; date +%s >> gpurun_out/r06_alive.txt; done ) &
HB=$!
trap "kill $HB" EXIT
W=5 S=20
echo "bench"
timeout -k 10 420 python bench.py --gpus 1 --steps $S --warmup $W > gpurun_out/r06_bench_all.json 2> gpurun_out/r06_bench_all.err \
  || { tail -20 gpurun_out/r06_bench_all.err; exit 1; }
echo "kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/r06_kt -o kt --output-format csv -- python bench.py --gpus 1 --steps $S --warmup $W \
  > gpurun_out/r06_kt_bench.json 2> gpurun_out/r06_kt.err || { tail -20 gpurun_out/r06_kt.err; exit 1; }
for f in $(find /tmp/r06_kt -name "*kernel_stats.csv"); do
  if grep -q k_leaf_step_ov $f; then cp $f gpurun_out/r06_bench_all_kernel_stats.csv; fi
  if grep -q igemm $f && ! grep -q k_leaf_step_ov $f; then cp $f gpurun_out/r06_bench_ppo_child_kernel_stats.csv; fi
done
TR=$(grep -l k_leaf_step_ov $(find /tmp/r06_kt -name "*kernel_trace.csv") | head -1)
python tools/window_avg.py $TR gpurun_out/r06_window_trace.json $W $S 100 256 \
  "round 6: rocprofv3 --kernel-trace of python bench.py --gpus 1 --steps $S --warmup $W (the driver's command), shipped build" || exit 1
rm -rf /tmp/r06_kt
ADDR=$(python -c "import json; print(int(json.load(open('gpurun_out/r06_bench_all.json'))['search_roofline']['addressed_bytes_per_sim_step']))")
echo "pmc selfplay (addressed $ADDR)"
tools/gpu/pmc_passes.sh /tmp/pmc_sp 300 -- python bench.py --workload selfplay --steps $S --warmup $W --no-cpu-baseline --late-plies 0 || exit 1
BK_PMC_RANGE=$((W*100)):$(((W+S)*100)) python tools/pmc_to_json.py gpurun_out/r06_pmc_selfplay.json k_leaf_step_ov k_leaf_step_ov 256 $ADDR \
  "round 6: rocprofv3 --pmc passes of bench.py --workload selfplay --steps $S --warmup $W (the driver's window): the mean over the window's k_leaf_step_ov dispatches ($((W*100))..$(((W+S)*100-1))); FETCH_SIZE x2 (gfx950); algorithmic_bytes = this build's search_roofline.addressed_bytes_per_sim_step (each W row per use)" /tmp/pmc_sp/p* || exit 1
python tools/pmc_to_json.py gpurun_out/r06_pmc_selfplay.json k_leafnet_x3 k_leafnet_x3 256 5677056 \
  "round 6: rocprofv3 --pmc passes of bench.py --workload selfplay --steps $S --warmup $W: the mean over every k_leafnet_x3 dispatch (256 boards, ResNet-5x64); algorithmic bytes = observations 3,276,800 + split weights 1,506,304 + pf/v out 823,296 (+ biases)" /tmp/pmc_sp/p* || exit 1
rm -rf /tmp/pmc_sp
echo "pmc legal"
tools/gpu/pmc_passes.sh /tmp/pmc_lg 200 -- python bench.py --workload legal --steps 20 --warmup 2 --no-cpu-baseline --graph 0 || exit 1
python tools/pmc_to_json.py gpurun_out/r06_pmc_legal.json k_legal_mask k_legal_mask 4096 17186816 \
  "round 6: rocprofv3 --pmc passes of bench.py --workload legal (eager launches, 4096 boards) on the shipped default k_legal_mask_rows<1,3,0,20>; algorithmic bytes = 4096 x (384 state + 3808 mask + 4 count)" /tmp/pmc_lg/p* || exit 1
rm -rf /tmp/pmc_lg
echo "pmc learner"
tools/gpu/pmc_passes.sh /tmp/pmc_ln 200 -- python tools/learner_pmc.py || exit 1
python tools/pmc_to_json.py gpurun_out/r06_pmc_learner.json k_conv_x3 "k_conv_x3(?!_)" 1024 209715200 \
  "round 6: rocprofv3 --pmc passes of tools/learner_pmc.py (the bench learner's main leg: batch 1024, 13 train steps + the kernel's own timing loop): every k_conv_x3 dispatch (forward and input gradient, 64->64 3x3, NHWC); algorithmic bytes = 1024 x (102,400 in + 102,400 out)" /tmp/pmc_ln/p* || exit 1
python tools/pmc_to_json.py gpurun_out/r06_pmc_learner.json k_conv_x3_wgrad "k_conv_x3_wgrad(?!_)" 1024 209862656 \
  "round 6: same passes: every k_conv_x3_wgrad dispatch (its reduce kernel not included); algorithmic bytes = 1024 x (102,400 x + 102,400 dy) + 147,456 dw (the partial-sum slabs are not algorithmic)" /tmp/pmc_ln/p* || exit 1
python tools/pmc_to_json.py gpurun_out/r06_pmc_learner.json k_bn_reduce k_bn_reduce 1024 157286400 \
  "round 6: same passes: the mean over every k_bn_reduce dispatch (the forward statistics read x: 104,857,600 B; the backward sums read dy and x: 209,715,200 B; as many of each)" /tmp/pmc_ln/p* || exit 1
python tools/pmc_to_json.py gpurun_out/r06_pmc_learner.json k_bn_axpb k_bn_axpb 1024 262144000 \
  "round 6: same passes: the mean over every k_bn_axpb dispatch (forward y = x s + t: 209,715,200 B; backward dx = dy k1 + k2 + x k3: 314,572,800 B; as many of each)" /tmp/pmc_ln/p* || exit 1
BK_PMC_SCALE=2 python tools/pmc_to_json.py gpurun_out/r06_pmc_learner.json "k_policy_loss+grad" k_policy_loss 1024 0 \
  "round 6: same passes: 2 x the mean over the k_policy_loss and k_policy_loss_grad dispatches = one launch pair; algorithmic bytes per pair: the bench line's bytes_per_launch_pair (K-dependent)" /tmp/pmc_ln/p* || exit 1
for k in k_splin_fwd k_splin_dx k_splin_dw; do
  python tools/pmc_to_json.py gpurun_out/r06_pmc_learner.json $k "$k(?!_)" 1024 0 \
    "round 6: same passes: every $k dispatch (the learner's policy Linear at the batch's legal ids, trainfc.hip); algorithmic bytes K-dependent (a 3.2-KB W or pf row per (row, legal id) pair from the Infinity Cache / L2, DESIGN section 4), so only the measured traffic is given" /tmp/pmc_ln/p* || exit 1
done
rm -rf /tmp/pmc_ln
echo ALLOK
