#!/bin/bash
# k_leafnet_x3p (8 waves, skewed halves) vs the 4-wave k_leafnet_x3 (BK_LN_W4=1): the leaf-net GPU
# tests, a bitwise A/B of the outputs, launch times interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/lnpp
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_leafnet_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 120 python tools/leafnet_ab.py dump $out/base.pt > $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
BK_LN_PP=1 timeout -k 10 120 python tools/leafnet_ab.py dump $out/new.pt >> $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
python tools/leafnet_ab.py cmp $out/base.pt $out/new.pt
for i in 1 2; do
  timeout -k 10 120 python tools/leafnet_bench.py 200 256 2>> $out/time.err | sed 's/^/w4 /' || exit 1
  BK_LN_PP=1 timeout -k 10 120 python tools/leafnet_bench.py 200 256 2>> $out/time.err | sed 's/^/pp /' || exit 1
done
