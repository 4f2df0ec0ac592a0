#!/bin/bash
# timing probe of the CGS2 inner GMRES variants (tools/variant_probe.sh SRC=krylov)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${PVARS:-base both}; do
  VAR=$v GS=${GS:-classical2} timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/probe_$v -o run -- python3 tools/inner_probe.py > gpurun_out/probe_$v.txt 2>&1 || exit 1
done
echo OK
