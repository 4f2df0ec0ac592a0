#!/bin/bash
# rocprofv3 kernel traces of the inner Schur GMRES (s-step) per timing variant:
#   VARS="old new" bash tools/ss_probe_prof.sh     (on the GPU box)
# runs tools/inner_probe.py on build/var/libdcp_<v>.so (tools/variant_probe.sh
# SRC=krylov builds them) into gpurun_out/ssp_<v>/ and gpurun_out/ssp_<v>.log.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in ${VARS:-base}; do
  VAR=$v GS=sstep timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ssp_$v -o run -- python3 tools/inner_probe.py > gpurun_out/ssp_$v.log 2>&1 || exit $?
done
