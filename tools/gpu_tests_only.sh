#!/bin/bash
# GPU parity suite only (K selects tests)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/t_gputest.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_gputest.log; exit 1; }
echo ALLOK
