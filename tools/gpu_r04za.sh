#!/bin/bash
# Constrained-diagonal pass on the second stream beside B^T + rhs (DCP_ASM_OVERLAP=3):
# assemble_nse_system timing (bitwise against mode 0), parity tests with it on
set -o pipefail
mkdir -p gpurun_out/r04za
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
REPS=16 timeout -k 10 300 python3 -u tools/env_probe.py DCP_ASM_OVERLAP 0 3 0 3 > gpurun_out/r04za/overlap3.json 2> gpurun_out/r04za/overlap3.err || { tail -5 gpurun_out/r04za/overlap3.err; exit 1; }
cat gpurun_out/r04za/overlap3.json
DCP_ASM_OVERLAP=3 timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_cube.py -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r04za/parity_tests_ov3.log 2>&1 || { echo "tests failed"; tail -15 gpurun_out/r04za/parity_tests_ov3.log; exit 1; }
tail -1 gpurun_out/r04za/parity_tests_ov3.log
