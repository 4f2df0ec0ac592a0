#!/bin/bash
# Nontemporal loads of read-once index streams: B^T task records (DCP_BT_NTLOAD,
# assembly timing, bitwise vs base) and the pencil's per-cell indices
# (DCP_MF_NTIDX, rocprofv3 stats of the matrix-free probe)
set -o pipefail
mkdir -p gpurun_out/r04zb
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
REPS=16 timeout -k 10 400 python3 -u tools/variant_probe.py > gpurun_out/r04zb/asm_variants.json 2> gpurun_out/r04zb/asm_variants.err || { tail -5 gpurun_out/r04zb/asm_variants.err; exit 1; }
cat gpurun_out/r04zb/asm_variants.json
VARS="a_base b_mfnt" timeout -k 10 500 bash tools/mf_variants.sh > gpurun_out/r04zb/mf_variants.txt 2>&1 || { echo "variants failed"; tail -5 gpurun_out/r04zb/mf_variants.txt; exit 1; }
cat gpurun_out/r04zb/mf_variants.txt
grep -h variant gpurun_out/mfvar/a_base.log gpurun_out/mfvar/b_mfnt.log
