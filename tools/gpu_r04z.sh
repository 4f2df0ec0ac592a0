#!/bin/bash
# Nontemporal B^T stores by default: operator-form / rhs / solve parity tests, the
# bench line; then matrix-free gather variants (GSPAN, GWAVES) by rocprofv3 stats
set -o pipefail
mkdir -p gpurun_out/r04z
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04z/parity_tests.log 2>&1 || { echo "tests failed"; tail -15 gpurun_out/r04z/parity_tests.log; exit 1; }
tail -1 gpurun_out/r04z/parity_tests.log
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04z/bench.json 2> gpurun_out/r04z/bench.err || { echo "bench failed"; tail -5 gpurun_out/r04z/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r04z/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['phase_ms'])"
VARS="a_base b_gs384 c_gs640 d_gw2 e_gw8" timeout -k 10 600 bash tools/mf_variants.sh > gpurun_out/r04z/mf_variants.txt 2>&1 || { echo "variants failed"; tail -5 gpurun_out/r04z/mf_variants.txt; exit 1; }
cat gpurun_out/r04z/mf_variants.txt
