#!/bin/bash
# the MFMA/VALU interleave probe, then the leaf-net epilogue-placement A/B (tools/gpu/epi_ab.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 5 60 ./tools/probe/mfma_epi || exit 1
bash tools/gpu/epi_ab.sh "$@"
