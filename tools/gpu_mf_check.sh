set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "matrix_free or operator or cube or multi_rank" > gpurun_out/t_mf.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_mf.log; exit 1; }
tail -2 gpurun_out/t_mf.log
rm -rf /tmp/pv; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pv -o run -- python3 tools/mf_probe.py > gpurun_out/mf_probe.log 2>&1 && find /tmp/pv -name "*kernel_stats.csv" -exec cp {} gpurun_out/mf_stats.csv \;
