#!/bin/bash
# B^T tasks beside the rhs launches on a second stream (DCP_ASM_OVERLAP): timing of
# assemble_nse_system per mode (bitwise against mode 0), then the operator-form
# parity tests with the overlap on
set -o pipefail
mkdir -p gpurun_out/r04x
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
REPS=16 timeout -k 10 300 python3 -u tools/env_probe.py DCP_ASM_OVERLAP 0 1 2 0 1 > gpurun_out/r04x/overlap.json 2> gpurun_out/r04x/overlap.err || { tail -5 gpurun_out/r04x/overlap.err; exit 1; }
cat gpurun_out/r04x/overlap.json
DCP_ASM_OVERLAP=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "operator_form or rhs or time_step or matches_oracle" \
  > gpurun_out/r04x/parity_tests_ov1.log 2>&1 || { echo "tests failed"; tail -15 gpurun_out/r04x/parity_tests_ov1.log; exit 1; }
tail -2 gpurun_out/r04x/parity_tests_ov1.log
