#!/bin/bash
# B^T task store variants (DCP_BT_STORE 0-3): assemble_nse_system at refine 5 per
# variant library, B^T and rhs bitwise against the first
set -o pipefail
mkdir -p gpurun_out/r04y
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
REPS=12 timeout -k 10 400 python3 -u tools/variant_probe.py > gpurun_out/r04y/bt_store_variants.json 2> gpurun_out/r04y/bt_store_variants.err || { tail -5 gpurun_out/r04y/bt_store_variants.err; exit 1; }
cat gpurun_out/r04y/bt_store_variants.json
