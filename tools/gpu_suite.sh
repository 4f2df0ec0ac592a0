#!/bin/bash
# Round GPU call: smoke, the parity suite, the default bench line and its
# rocprofv3 kernel statistics; TAG names the outputs (gpurun_out/TAG_*).
set -o pipefail
TAG=${TAG:-r05}
tools/gpu_job.sh ${TAG}_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" &&
tools/gpu_job.sh ${TAG}_gputest 1100 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=20 &&
tools/gpu_job.sh ${TAG}_bench 600 python3 bench.py &&
tools/gpu_job.sh ${TAG}_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
