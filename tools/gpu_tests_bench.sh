#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/s2_gputest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/s2_gputest.log; exit 1; }
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/s2_bench.json 2> gpurun_out/s2_bench.err || { echo "bench failed"; tail -5 gpurun_out/s2_bench.err; exit 1; }
echo ALLOK
