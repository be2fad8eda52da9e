#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
for m in zero center shift normal; do
timeout -k 10 120 python tools/leafnet_debug.py $m 2>&1 | grep -v amdgpu.ids || exit 1
done
