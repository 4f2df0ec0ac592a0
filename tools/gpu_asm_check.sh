#!/bin/bash
# Assembly change check: the parity tests that read B / B^T, then the r=5
# assembly timing (tools/asm_probe.py) under rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${K:-operator or golden or parity_gpu or cube or multi_rank}" > gpurun_out/t_asm.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_asm.log; exit 1; }
tail -2 gpurun_out/t_asm.log
rm -rf /tmp/pa
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pa -o run -- python3 tools/asm_probe.py > gpurun_out/asm_probe.log 2>&1 && find /tmp/pa -name "*kernel_stats.csv" -exec cp {} gpurun_out/asm_stats.csv \;
grep variant gpurun_out/asm_probe.log
