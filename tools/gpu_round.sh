#!/bin/bash
# One GPU call: parity suite, default bench line, rocprofv3 kernel stats of the bench.
# TAG names the outputs (profiles/<TAG>_*).
set -o pipefail
TAG=${TAG:-r02}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=15 > gpurun_out/${TAG}_gputest.log 2>&1 || { echo "tests failed"; tail -5 gpurun_out/${TAG}_gputest.log; exit 1; }
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench_prof.json 2> gpurun_out/${TAG}_prof.err || { echo "prof failed"; tail -5 gpurun_out/${TAG}_prof.err; exit 1; }
echo ALLOK
