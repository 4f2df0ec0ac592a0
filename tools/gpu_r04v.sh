#!/bin/bash
# Pencil LDS aliasing (DCP_MF_LDS_ALIAS): matrix-free / rhs parity tests, then the
# alias / no-alias A/B (rocprofv3 kernel stats of tools/mf_probe.py per variant)
set -o pipefail
mkdir -p gpurun_out/r04v
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "matrix_free or operator_form or operator_applies or rhs or time_step or smoke" \
  > gpurun_out/r04v/parity_tests.log 2>&1 || { echo "tests failed"; tail -15 gpurun_out/r04v/parity_tests.log; exit 1; }
tail -2 gpurun_out/r04v/parity_tests.log
VARS="alias noalias" timeout -k 10 500 bash tools/mf_variants.sh > gpurun_out/r04v/mf_variants.txt 2>&1 || { echo "variants failed"; tail -5 gpurun_out/r04v/mf_variants.txt; exit 1; }
cat gpurun_out/r04v/mf_variants.txt
grep -h "variant" gpurun_out/mfvar/*.log
