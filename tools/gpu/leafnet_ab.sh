#!/bin/bash
# k_leafnet_x3 change check: its GPU tests, a bitwise A/B against a saved earlier build
# (blokus_rl_amd/_lib/exp/libbase.so), the launch timing and the phase stamps of the new build.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/ab
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_leafnet_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
# reference outputs: a dump of an earlier build (blokus_rl_amd/_lib/exp/ref.pt), else libbase.so
if [ -f blokus_rl_amd/_lib/exp/ref.pt ]; then
  cp blokus_rl_amd/_lib/exp/ref.pt $out/base.pt
else
  BK_LIB=blokus_rl_amd/_lib/exp/libbase.so timeout -k 10 120 python tools/leafnet_ab.py dump $out/base.pt > $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
fi
timeout -k 10 120 python tools/leafnet_ab.py dump $out/new.pt >> $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
python tools/leafnet_ab.py cmp $out/base.pt $out/new.pt
[ -f blokus_rl_amd/_lib/exp/libbase.so ] && { BK_LIB=blokus_rl_amd/_lib/exp/libbase.so timeout -k 10 120 python tools/leafnet_bench.py 200 256 2> $out/time.err || exit 1; }
timeout -k 10 120 python tools/leafnet_bench.py 200 256 2>> $out/time.err || exit 1
if [ -f blokus_rl_amd/_lib/exp/libln_st.so ]; then
  BK_LIB=blokus_rl_amd/_lib/exp/libln_st.so timeout -k 10 120 python tools/leafnet_bench.py 50 256 --stamps 2>> $out/time.err || exit 1
fi
