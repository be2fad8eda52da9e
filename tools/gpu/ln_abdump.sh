cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/ab; mkdir -p $out
BK_LIB=blokus_rl_amd/_lib/exp/libbase.so timeout -k 10 120 python tools/leafnet_ab.py dump $out/base.pt > $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
timeout -k 10 120 python tools/leafnet_ab.py dump $out/new.pt >> $out/dump.log 2>&1 || { tail $out/dump.log; exit 1; }
python tools/leafnet_ab.py cmp $out/base.pt $out/new.pt
exit 0
