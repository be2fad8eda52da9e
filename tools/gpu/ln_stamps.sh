cd "$GRAFT_REPO_ROOT" && BK_LIB=blokus_rl_amd/_lib/exp/liblnst.so timeout -k 10 120 python tools/leafnet_bench.py 50 256 --stamps
