#!/bin/bash
# Learner framework-level A/B (tools/learner_ab.py): ms per Adam step at batch 1024 and 64.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/learner_ab.py --batch 1024 --steps 20 > gpurun_out/learner_ab.jsonl 2> gpurun_out/learner_ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/learner_ab.jsonl; tail -3 gpurun_out/learner_ab.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/learner_ab.py --batch 64 --steps 40 --configs base,nativebn,cl+nativebn > gpurun_out/learner_ab64.jsonl 2>> gpurun_out/learner_ab.err
rc=$?; echo "ab64 rc=$rc"; cat gpurun_out/learner_ab64.jsonl
exit $rc
