#!/bin/bash
# CGS2 parity subset + r=5 bench lines in both Gram-Schmidt modes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "classical2 or CGS2 or cgs2 or operator_form" > gpurun_out/cgs2_test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/cgs2_test.log; exit 1; }
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gram-schmidt classical2 > gpurun_out/cgs2_bench.json 2> gpurun_out/cgs2_bench.err || { echo "bench failed"; tail -5 gpurun_out/cgs2_bench.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/cgs2_prof -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --gram-schmidt classical2 > gpurun_out/cgs2_bench_prof.json 2> gpurun_out/cgs2_prof.err || { echo "prof failed"; tail -5 gpurun_out/cgs2_prof.err; exit 1; }
echo ALLOK
