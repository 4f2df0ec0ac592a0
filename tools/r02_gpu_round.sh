#!/bin/bash
# One GPU call: parity suite, default bench line, rocprofv3 kernel stats of the bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r02_gputest.log 2>&1 || { echo "tests failed"; tail -5 gpurun_out/r02_gputest.log; exit 1; }
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || { echo "bench failed"; tail -5 gpurun_out/r02_bench.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02_bench_prof.json 2> gpurun_out/r02_prof.err || { echo "prof failed"; tail -5 gpurun_out/r02_prof.err; exit 1; }
echo ALLOK
