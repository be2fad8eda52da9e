#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so timeout -k 10 300 python tools/stamp_step.py 6
